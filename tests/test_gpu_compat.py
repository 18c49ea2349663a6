"""Reference-compatible module API on the HIP device (cbf.CBF / controller.Controller forward
through the native autograd Functions) against autograd through the fp32 oracle."""
import math

import pytest
import torch

import core
from macbf_gnn_amd import config as C
from macbf_gnn_amd import oracle as O
from macbf_gnn_amd.models import CBF, Controller

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


def _cmp(got, ref, name, rel=0.1, cos=0.99):
    got, ref = got.double().flatten(), ref.double().flatten()
    rn = ref.norm().item()
    if rn < 1e-12:
        assert got.norm().item() < 1e-6, name
        return
    err = (got - ref).norm().item() / rn
    c = torch.nn.functional.cosine_similarity(got, ref, dim=0).item()
    assert err < rel and c > cos, f"{name}: rel {err:.3e} cos {c:.5f}"


@pytest.mark.parametrize("B,N", [(1, 8), (2, 40), (1, 300)])
def test_cbf_module_forward_backward(B, N):
    torch.manual_seed(1)
    cbf = _round_bf16(CBF(4).to(DEV))
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
    href = O.cbf_forward(p, s2, idx)
    gr = torch.autograd.grad((href * w).sum(), [s2] + list(p.values()))
    _cmp(h.detach(), href.detach(), "h", rel=3e-2, cos=0.999)
    _cmp(sx.grad, gr[0], "dL/ds")
    tol = 0.15 if B * N * K < 1000 else 0.1      # tiny graphs: fewer edges to average bf16 noise over
    for (k, prm), ref in zip(cbf.named_parameters(), gr[1:]):
        _cmp(prm.grad, ref, k, rel=tol)


@pytest.mark.parametrize("B,N", [(1, 8), (2, 64)])
def test_controller_module_forward_backward(B, N):
    torch.manual_seed(2)
    ctrl = _round_bf16(Controller(4).to(DEV))
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
    aref = O.controller_forward(p, s2, g, idx)
    gr = torch.autograd.grad((aref * w).sum(), [s2] + list(p.values()))
    _cmp(a.detach(), aref.detach(), "a", rel=3e-2, cos=0.999)
    _cmp(sx.grad, gr[0], "dL/ds")
    tol = 0.15 if B * N < 100 else 0.1
    for (k, prm), ref in zip(ctrl.named_parameters(), gr[1:]):
        _cmp(prm.grad, ref, k, rel=tol)


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
