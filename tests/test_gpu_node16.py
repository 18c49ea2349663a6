"""The 16x16x32 x3 node backward (csrc/node16.h: 16 agents per wave, two waves per SIMD).

* a full training step with the kernel forced on (128-agent node chunks at small sizes) against
  autograd through the fp32 oracle engine: every parameter gradient <= 1e-3 relative;
* the BPTT recursion (G_t, dL/dpooled, ego terms) and the gradients against the 32x32x16 node kernel
  on the same step (both fp32-accurate split-bf16, different accumulation orders).
Reference op: /root/reference/controller.py:23-29,47-61 differentiated by /root/reference/train.py:103.
"""
import pytest
import torch

from macbf_gnn_amd import config as C
from macbf_gnn_amd.ops import native

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _trainer(**kw):
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.parallel import DP
    cfg = C.TrainConfig(num_agents=kw.pop("N"), num_envs=kw.pop("B"), inner_loops=kw.pop("T", 5), early_stop=False,
                        seed=kw.pop("seed", 0), device="hip", dtype="fp32", **kw)
    return Trainer(cfg, device=DEV, dp=DP(device=DEV))


def _rel(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float((a - b).norm() / b.norm().clamp(min=1e-30))


@pytest.mark.parametrize("native_bptt", [True, False])
@pytest.mark.parametrize("N,B,extra", [(256, 2, {}), (13, 5, {}), (64, 3, dict(dim=3, num_obstacles=2)),
                                       (200, 3, dict(reuse_nbr_idx=False))])
def test_node16_full_step_vs_oracle(N, B, extra, native_bptt, monkeypatch):
    from macbf_gnn_amd.engine.hip_engine import HipEngine
    from macbf_gnn_amd.engine.oracle_engine import OracleEngine
    monkeypatch.setattr(HipEngine, "native_bptt", native_bptt)
    monkeypatch.setenv("MACBF_NODE_CHUNK", "128")
    monkeypatch.setenv("MACBF_BWD_FUSED", "0")
    tr = _trainer(N=N, B=B, **extra)
    assert tr.engine._node16(B * N) is not None
    s0, g, obs = tr.sample()
    tr.engine.step(s0, g, obs)
    g_hip = tr.fp.grad.clone()
    OracleEngine(tr).step(s0, g, obs)
    g_ref = tr.fp.grad.clone()
    worst = sorted(((_rel(g_hip[o:o + n], g_ref[o:o + n]), pn) for m, pn, shape, o, n in tr.fp.specs), reverse=True)
    assert worst[0][0] <= 1e-3, worst[:4]


@pytest.mark.parametrize("N,B,extra", [(1024, 2, {}), (96, 3, dict(dim=3, num_obstacles=1))])
def test_node16_matches_node32(N, B, extra, monkeypatch):
    monkeypatch.setenv("MACBF_NODE_CHUNK", "128")
    monkeypatch.setenv("MACBF_BWD_FUSED", "0")
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("MACBF_NODE16", mode)
        tr = _trainer(N=N, B=B, T=8, **extra)
        assert (tr.engine._node16(B * N) is not None) == (mode == "1")
        s0, g, obs = tr.sample()
        tr.engine.step(s0, g, obs)
        torch.cuda.synchronize()
        e = tr.engine
        out[mode] = (e.Gb.clone(), e.dP.clone(), e.ego.clone(), tr.fp.grad.clone(), tr.fp.specs)
    new, old = out["1"], out["0"]
    assert torch.isfinite(new[0]).all() and torch.isfinite(new[3]).all()
    assert _rel(new[0], old[0]) <= 1e-4, _rel(new[0], old[0])          # G_t recursion
    dpn = new[1][..., :128].float() + new[1][..., 128:].float()         # dL/dpooled = hi + lo planes
    dpo = old[1][..., :128].float() + old[1][..., 128:].float()
    assert _rel(dpn, dpo) <= 1e-4, _rel(dpn, dpo)
    assert _rel(new[2], old[2]) <= 1e-4
    for m, pn, shape, o, n in new[4]:
        if m == "controller":
            assert _rel(new[3][o:o + n], old[3][o:o + n]) <= 1e-4, pn


@pytest.mark.parametrize("dtype,extra", [("bf16", {}), ("fp16", {}), ("bf16", dict(dim=3, num_obstacles=2)),
                                         ("fp16", dict(dim=3, num_obstacles=2))])
def test_node16_matches_node32_1pass(dtype, extra, monkeypatch):
    """The 1-pass builds (round 4: the 16x16x32 node backward is their default at 128-agent chunks;
    config #5 runs it in fp16 with 3-D states and obstacle nodes -- ADVICE r4): same step against the
    32x32x16 kernel. Both round the activations to 16 bits at the same points;
    accumulation orders differ, so a rounding can flip: bounds of the bf16 full-step tests (2e-2)."""
    monkeypatch.setenv("MACBF_NODE_CHUNK", "128")
    monkeypatch.setenv("MACBF_BWD_FUSED", "0")
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("MACBF_NODE16", mode)
        from macbf_gnn_amd.engine import Trainer
        from macbf_gnn_amd.parallel import DP
        cfg = C.TrainConfig(num_agents=256, num_envs=2, inner_loops=8, early_stop=False, seed=0, device="hip",
                            dtype=dtype, **extra)
        tr = Trainer(cfg, device=DEV, dp=DP(device=DEV))
        assert (tr.engine._node16(2 * 256) is not None) == (mode == "1")
        s0, g, obs = tr.sample()
        tr.engine.step(s0, g, obs)
        torch.cuda.synchronize()
        out[mode] = (tr.engine.Gb.clone(), tr.engine.dP.float().clone(), tr.fp.grad.clone(), tr.fp.specs)
    new, old = out["1"], out["0"]
    assert torch.isfinite(new[0]).all() and torch.isfinite(new[2]).all()
    assert _rel(new[0], old[0]) <= 2e-2, _rel(new[0], old[0])
    assert _rel(new[1], old[1]) <= 2e-2, _rel(new[1], old[1])
    for m, pn, shape, o, n in new[3]:
        if m == "controller":
            assert _rel(new[2][o:o + n], old[2][o:o + n]) <= 2e-2, pn


@pytest.mark.parametrize("dtype,dim", [("fp32", 2), ("bf16", 2), ("fp16", 3)])
def test_node16_startup_selfcheck(dtype, dim, monkeypatch):
    """ops.selfcheck runs the 16x16x32 node backward against the 32x32x16 one when an engine that
    uses it is built, in every precision; a corrupted weight image is caught."""
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.ops import selfcheck
    from macbf_gnn_amd.parallel import DP
    monkeypatch.setenv("MACBF_NODE_CHUNK", "128")
    monkeypatch.setenv("MACBF_BWD_FUSED", "0")
    cfg = C.TrainConfig(num_agents=256, num_envs=2, inner_loops=4, seed=0, device="hip", dtype=dtype, dim=dim)
    tr = Trainer(cfg, device=DEV, dp=DP(device=DEV))
    rep = tr.engine.selfcheck
    assert rep and rep["node16"]["worst_rel"] <= rep["node16"]["tol"], rep
    w = tr.engine.node16_w
    keep = w.clone()
    w.view(-1)[64 * 176: 64 * 176 + 4096] = 0            # W2 rows of the hi plane
    with pytest.raises(native.NativeError):
        selfcheck.check(tr.engine)
    w.copy_(keep)
    assert selfcheck.check(tr.engine)["node16"]["worst_rel"] <= rep["node16"]["tol"]
