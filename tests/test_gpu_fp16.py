"""fp16 mixed precision (BASELINE config #5): the fp16 instantiation of the
controller / CBF kernels (csrc/prec.h) with dynamic loss scaling, against the fp32 oracle."""
import pytest
import torch

from macbf_gnn_amd import config as C
from macbf_gnn_amd.ops import native

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _cmp(got, ref, name, rel=0.12, cos=0.99):
    got, ref = got.double().flatten(), ref.double().flatten()
    rn = ref.norm().item()
    err = (got - ref).norm().item() / max(rn, 1e-12)
    c = torch.nn.functional.cosine_similarity(got, ref, dim=0).item()
    assert err < rel and c > cos, f"{name}: rel {err:.3e} cos {c:.5f}"


def _trainer(**kw):
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.parallel import DP
    cfg = C.TrainConfig(num_agents=kw.pop("N", 48), num_envs=kw.pop("B", 2), inner_loops=kw.pop("T", 5),
                        early_stop=kw.pop("early_stop", False), seed=0, device="hip", dtype="fp16", **kw)
    return Trainer(cfg, device=DEV, dp=DP(device=DEV))


def test_fp16_weights_and_buffers_are_half():
    tr = _trainer()
    assert tr.fp16 and tr.grad_scale == C.TrainConfig().loss_scale_init
    pw = tr.engine.pw
    for t in (pw.ctrl_w, pw.cbf_w, pw.ctrl_rm, pw.cbf_rm, tr.engine.pooled, tr.engine.dP):
        assert t.dtype == torch.float16


@pytest.mark.parametrize("dim,nobs,bptt", [(2, 0, True), (3, 3, True), (3, 3, False)])
def test_fp16_full_step_matches_oracle(dim, nobs, bptt):
    """One full fp16 training step (scaled upstream gradients, unscaled flat gradient) vs
    autograd through the fp32 oracle."""
    from macbf_gnn_amd.engine.oracle_engine import OracleEngine
    tr = _trainer(dim=dim, num_obstacles=nobs, bptt=bptt)
    s0, g, obs = tr.sample()
    stats = tr.engine.step(s0, g, obs)
    g_hip = tr.fp.grad.clone()
    assert torch.isfinite(g_hip).all()
    stats_o = OracleEngine(tr).step(s0, g, obs)
    g_ref = tr.fp.grad.clone()
    for name in ("controller", "cbf"):
        a_, b_ = tr.fp.ranges[name]
        _cmp(g_hip[a_:b_], g_ref[a_:b_], name)
    assert abs(float(stats["loss_total"]) - stats_o["loss_total"]) <= 0.05 * abs(stats_o["loss_total"]) + 1e-4


def test_fp16_gradient_is_scale_invariant():
    """The loss scale only moves the fp16 operating range: grads at scales 512 and 4096 agree."""
    tr = _trainer(N=64, B=2)
    s0, g, obs = tr.sample()
    tr.grad_scale = 4096.0
    tr.engine.step(s0, g, obs)
    g1 = tr.fp.grad.clone()
    tr.grad_scale = 512.0
    tr.engine.step(s0, g, obs)
    _cmp(tr.fp.grad, g1, "scale", rel=0.03, cos=0.999)


def test_fp16_overflow_skips_step_and_backs_off():
    tr = _trainer(N=32, B=1, T=4)
    before = tr.fp.flat.clone()
    tr.grad_scale = 2.0 ** 24          # forces fp16 overflow in the backward deltas
    st = tr.train_step()
    torch.cuda.synchronize()
    if st.get("skipped"):
        assert tr.grad_scale == 2.0 ** 23 and torch.equal(before, tr.fp.flat)
    for _ in range(20):                # the scale halves per skipped step until the step is finite
        st = tr.train_step()
    torch.cuda.synchronize()
    assert tr.grad_scale < 2.0 ** 23 and not st.get("skipped")
    assert torch.isfinite(tr.fp.flat).all() and not torch.equal(before, tr.fp.flat)


def test_fp16_module_api():
    """Reference-module API with fp16 packed weights (``mfma_dtype`` attribute), fwd + bwd."""
    from macbf_gnn_amd import env as E
    from macbf_gnn_amd import oracle as O
    from macbf_gnn_amd.models import CBF, Controller
    torch.manual_seed(0)
    cbf, ctrl = CBF(4).to(DEV), Controller(4).to(DEV)
    cbf.mfma_dtype = ctrl.mfma_dtype = torch.float16
    s, g = E.generate_batch(2, 40, seed=2)
    s[..., 2:] = 0.3 * torch.randn_like(s[..., 2:])
    s, g = s.to(DEV), g.to(DEV)
    idx = O.knn_idx(s, C.TOP_K)
    sx = s.clone().requires_grad_(True)
    h = cbf(sx)
    a = ctrl(s, g)
    (h.sum() + a.square().sum()).backward()
    p = {k: v.detach().clone().requires_grad_(True) for k, v in cbf.params_dict().items()}
    s2 = s.clone().requires_grad_(True)
    href = O.cbf_forward(p, s2, idx)
    gs, gw = torch.autograd.grad(href.sum(), [s2, p["cbf_net.2.weight"]])
    _cmp(h.detach(), href.detach(), "h", rel=0.03, cos=0.999)
    _cmp(sx.grad, gs, "dh/ds", rel=0.1)
    _cmp(cbf.cbf_net[2].weight.grad, gw, "dh/dW2", rel=0.1)
    _cmp(a.detach(), O.controller_forward(ctrl.params_dict(), s, g, idx), "actions", rel=0.03, cos=0.999)


def test_fp16_kernel_variant_is_loaded():
    lib = native.lib()
    for n in ("ctrl_fwd", "cbf_bwd", "ctrl_node_bwd", "ctrl_edge_bwd"):
        assert hasattr(lib, n)
