"""Reference-compatible module API on the HIP device (cbf.CBF / controller.Controller forward
through the native autograd Functions) against autograd through the oracle: the default fp32
(x3) kernels vs the fp32 oracle, and the bf16 kernels (``mfma_dtype = torch.bfloat16``, bf16
weights) vs the oracle in bf16-emulation mode."""
import math

import pytest
import torch

import core
from macbf_gnn_amd import config as C
from macbf_gnn_amd import oracle as O
from macbf_gnn_amd.models import CBF, Controller
from numerics import ctrl_pool_slots, rel_cmp

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _round_bf16(m):
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(p.bfloat16().float())
    return m


def _states(B, N, seed, vscale=0.6):
    g = torch.Generator().manual_seed(seed)
    L = math.sqrt(max(1.0, N / 8.0)) * 0.7
    p = torch.rand(B, N, 2, generator=g) * L
    v = (torch.rand(B, N, 2, generator=g) - 0.5) * 2 * vscale
    goals = p + (torch.rand(B, N, 2, generator=g) - 0.5)
    return torch.cat([p, v], -1).to(DEV), goals.to(DEV)


def _cmp(got, ref, name, rel):
    rel_cmp(got, ref, name, rel)


# (forward, gradient) relative-norm bounds per precision; bf16 against the emulating oracle
TOL = {"fp32": (1e-4, 1e-3), "bf16": (1e-2, 2e-2)}
# the kernels' argmax slots are maxima up to near-ties of this relative size
SLOT_GAP = {"fp32": 1e-5, "bf16": 1e-4}


def _prec(m, prec):
    if prec == "bf16":
        m.mfma_dtype = torch.bfloat16
        _round_bf16(m)
    return m


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("B,N", [(1, 8), (2, 40), (1, 300)])
def test_cbf_module_forward_backward(B, N, prec):
    torch.manual_seed(1)
    cbf = _prec(CBF(4).to(DEV), prec)
    tf, tg = TOL[prec]
    s, _ = _states(B, N, seed=N)
    K = min(N, C.TOP_K)
    idx = O.knn_idx(s, K)
    sx = s.clone().requires_grad_(True)
    h = cbf(sx)
    assert h.shape == (B, N, K)
    w = torch.randn_like(h)
    (h * w).sum().backward()
    p = {k: v.detach().clone().requires_grad_(True) for k, v in cbf.params_dict().items()}
    s2 = s.clone().requires_grad_(True)
    with O.emulate_bf16(prec == "bf16"):
        href = O.cbf_forward(p, s2, idx)
        gr = torch.autograd.grad((href * w).sum(), [s2] + list(p.values()))
    _cmp(h, href, "h", rel=tf)
    _cmp(sx.grad, gr[0], "dL/ds", rel=tg)
    for (k, prm), ref in zip(cbf.named_parameters(), gr[1:]):
        _cmp(prm.grad, ref, k, rel=tg)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("B,N", [(1, 8), (2, 64)])
def test_controller_module_forward_backward(B, N, prec):
    torch.manual_seed(2)
    ctrl = _prec(Controller(4).to(DEV), prec)
    tf, tg = TOL[prec]
    s, g = _states(B, N, seed=N + 1)
    K = min(N, C.TOP_K)
    idx = O.knn_idx(s, K)
    sx = s.clone().requires_grad_(True)
    a = ctrl(sx, g)
    assert a.shape == (B, N, 2)
    w = torch.randn_like(a)
    (a * w).sum().backward()
    p = {k: v.detach().clone().requires_grad_(True) for k, v in ctrl.params_dict().items()}
    s2 = s.clone().requires_grad_(True)
    slots, pvals = ctrl_pool_slots(ctrl, s, g, idx)
    with O.emulate_bf16(prec == "bf16"):
        aref, aux = O.controller_forward(p, s2, g, idx, return_aux=True, pool_slots=slots, pool_values=pvals)
        gr = torch.autograd.grad((aref * w).sum(), [s2] + list(p.values()))
    assert O.pool_slot_gap(aux["hm"].detach(), slots) < SLOT_GAP[prec]
    with O.emulate_bf16(prec == "bf16"):       # forward checks: the oracle's own max-pool
        afree, aux_f = O.controller_forward(p, s, g, idx, return_aux=True)
    _cmp(pvals, aux_f["pooled"], "pooled", rel=tf)
    _cmp(a, afree, "a", rel=tf)
    _cmp(sx.grad, gr[0], "dL/ds", rel=tg)
    for (k, prm), ref in zip(ctrl.named_parameters(), gr[1:]):
        _cmp(prm.grad, ref, k, rel=tg)


def test_core_api_on_device():
    """core.py entry points (single env, reference shapes) run on the device and backprop."""
    torch.manual_seed(0)
    ctrl, cbf = Controller(4).to(DEV), CBF(4).to(DEV)
    s, g = _states(1, 32, seed=3)
    s, g = s[0], g[0]
    a = ctrl(s, g)
    h = cbf(s)
    assert a.shape == (32, 2) and h.shape == (32, 1, 12)
    lb = core.loss_barrier(h, s)
    ld = core.loss_derivatives(s, a, h, cbf)
    la = core.loss_actions(s, g, a)
    total = sum(lb[:2]) + sum(ld[:2]) + la
    total.backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in ctrl.parameters())
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in cbf.parameters())


def test_evaluate_with_refinement_on_device():
    from macbf_gnn_amd.evaluate import EvalConfig, evaluate
    torch.manual_seed(3)
    m = evaluate(Controller(4).to(DEV), CBF(4).to(DEV),
                 EvalConfig(num_agents=64, num_envs=2, episodes=1, max_steps=4, refine_loops=3), device=DEV)
    assert 0.0 <= m["safety_rate"] <= 1.0 and m["agent_steps"] > 0
