"""Persistent small-scene rollout (csrc/ctrl.hip rollout_small_kernel): one launch for the whole
rollout, one workgroup per env, device-side early stop. It must reproduce the launch-per-step
native driver bit for bit: horizon, trajectories, kNN graphs, danger bits, counts, safety, actions,
per-env sums, pooled features / argmax slots, and the training gradient."""
import pytest
import torch

from macbf_gnn_amd import config as C
from macbf_gnn_amd.ops import native

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _trainer(small, **kw):
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.engine.hip_engine import HipEngine
    from macbf_gnn_amd.parallel import DP
    cfg = C.TrainConfig(num_agents=kw.pop("N", 32), num_envs=kw.pop("B", 4), inner_loops=kw.pop("T", 40),
                        seed=kw.pop("seed", 3), device="hip", **kw)
    old = HipEngine.small_rollout
    HipEngine.small_rollout = small
    try:
        tr = Trainer(cfg, device=DEV, dp=DP(device=DEV))
    finally:
        HipEngine.small_rollout = old
    assert tr.engine.small_rollout == (small and tr.engine.Nn <= 64)
    return tr


def _outputs(tr, s0, g, obs, early_stop):
    eng = tr.engine
    T = eng.rollout(s0, g, obs, early_stop=early_stop)
    torch.cuda.synchronize()
    out = dict(S=eng.S[: T + 1], idx=eng.idx[:T], dang=eng.dang[:T], cnt=eng.cnt[:T], A=eng.A[:T],
               dist=eng.dist[:T], act=eng.act[:T], pooled=eng.pooled[:T], argmax=eng.argmax[:T])
    if tr.cfg.compute_safety:
        out["safe"] = eng.safe[: T + 1]
    return T, {k: v.clone() for k, v in out.items()}


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("early_stop", [True, False])
def test_small_rollout_matches_per_step_driver(dtype, early_stop):
    a, b = _trainer(False, dtype=dtype), _trainer(True, dtype=dtype)
    b.fp.flat.copy_(a.fp.flat)
    b.engine.after_update()
    s0, g, obs = a.sample()
    Ta, oa = _outputs(a, s0, g, obs, early_stop)
    Tb, ob = _outputs(b, s0, g, obs, early_stop)
    assert Ta == Tb
    if early_stop:
        assert Ta < a.cfg.inner_loops
    for k in oa:
        assert torch.equal(oa[k], ob[k]), k


@pytest.mark.parametrize("kw", [dict(dim=3, num_obstacles=2, N=24), dict(N=64, B=2), dict(N=10, B=5),
                                dict(N=32, B=3, add_noise_prob=0.5, noise_scale=0.3)])
def test_small_rollout_variants(kw):
    """3-D with obstacle nodes (Nn = 24 + 24), a full 64-node env, an odd agent count, and the
    device exploration noise (keyed by the global env index)."""
    a, b = _trainer(False, T=25, **kw), _trainer(True, T=25, **kw)
    b.fp.flat.copy_(a.fp.flat)
    b.engine.after_update()
    s0, g, obs = a.sample()
    Ta, oa = _outputs(a, s0, g, obs, True)
    Tb, ob = _outputs(b, s0, g, obs, True)
    assert Ta == Tb
    for k in oa:
        assert torch.equal(oa[k], ob[k]), k


def test_small_rollout_training_step_matches():
    a, b = _trainer(False, T=20), _trainer(True, T=20)
    # bit-for-bit: the stored node activations round the backward differently from the per-step
    # recompute (covered with a tolerance by test_gpu_runtime's node-activation test)
    b.engine.node_acts = None
    b.fp.flat.copy_(a.fp.flat)
    b.engine.after_update()
    s0, g, obs = a.sample()
    sa = a.engine.step(s0, g, obs)
    sb = b.engine.step(s0, g, obs)
    assert float(sa["T"]) == float(sb["T"])
    assert torch.equal(a.fp.grad, b.fp.grad)


def test_small_rollout_repeatable_and_trains():
    tr = _trainer(True, T=30, B=6)
    s0, g, obs = tr.sample()
    T1, o1 = _outputs(tr, s0, g, obs, True)
    T2, o2 = _outputs(tr, s0, g, obs, True)
    assert T1 == T2
    for k in o1:
        assert torch.equal(o1[k], o2[k]), k
    before = tr.fp.flat.clone()
    for _ in range(3):
        st = tr.train_step()
    torch.cuda.synchronize()
    assert torch.isfinite(tr.fp.flat).all() and not torch.equal(before, tr.fp.flat)
    assert float(st["agent_steps"]) > 0


@pytest.mark.parametrize("native_bptt,N,B", [(True, 256, 8), (False, 256, 8), (True, 1024, 12), (False, 1024, 12)])
def test_fused_bptt_step_matches_separate_launches(native_bptt, N, B, monkeypatch):
    """Fused node + edge backward per reverse step (csrc/ctrl.hip ctrl_bwd_step_kernel, the
    strong-scaling slice path) against the separate node / edge launches: the recursion (G, dP,
    ego) bit for bit; the weight gradients up to the slab summation order (the edge slab rows
    differ). The separate launches use the 32x32x16 edge backward (MACBF_EB16=0), whose body the
    fused step shares. 1024 x 12 agents: 384 32-agent chunks on a grid of one workgroup per CU, so
    workgroups run a second node chunk while others already write step t's edge records (the
    double-buffered dEc keeps step t+1's records intact)."""
    from macbf_gnn_amd.engine.hip_engine import HipEngine
    monkeypatch.setattr(HipEngine, "native_bptt", native_bptt)
    monkeypatch.setenv("MACBF_EB16", "0")
    trs = []
    for fused in ("0", "1"):
        monkeypatch.setenv("MACBF_BWD_FUSED", fused)
        trs.append(_trainer(False, N=N, B=B, T=12))
    a, b = trs
    assert b.engine.nb_node == b.engine.nb_edge
    assert native.bwd_step_fused(B * N, b.engine.dev) and native.node_bwd_chunk(B * N, b.engine.dev) == 32
    b.fp.flat.copy_(a.fp.flat)
    b.engine.after_update()
    s0, g, obs = a.sample()
    monkeypatch.setenv("MACBF_BWD_FUSED", "0")
    a.engine.step(s0, g, obs)
    monkeypatch.setenv("MACBF_BWD_FUSED", "1")
    b.engine.step(s0, g, obs)
    torch.cuda.synchronize()
    assert torch.equal(a.engine.Gb, b.engine.Gb)
    assert torch.equal(a.engine.dP, b.engine.dP) and torch.equal(a.engine.ego, b.engine.ego)
    torch.testing.assert_close(b.fp.grad, a.fp.grad, rtol=2e-5, atol=1e-8)


@pytest.mark.parametrize("kw", [dict(dtype="fp32"), dict(dtype="bf16", N=32, B=1), dict(dtype="fp16", N=20, B=3),
                                dict(dtype="fp32", dim=3, num_obstacles=2, N=24)])
def test_backward_graph_matches_eager(kw, monkeypatch):
    """Small scenes: the post-rollout work (counts, CBF losses + backward, BPTT, gradient assembly)
    replayed from a HIP graph captured per horizon T gives the eager step's gradient and statistics
    bit for bit -- the first occurrence of a T runs eagerly and captures, later ones replay."""
    monkeypatch.setenv("MACBF_BWD_GRAPH", "0")
    a = _trainer(True, T=20, **dict(kw))
    monkeypatch.setenv("MACBF_BWD_GRAPH", "1")
    b = _trainer(True, T=20, **dict(kw))
    assert b.engine._bwd_graph_on() and not a.engine._bwd_graph_on()
    b.fp.flat.copy_(a.fp.flat)
    b.engine.after_update()
    s0, g, obs = a.sample()
    for it in range(3):
        sa = a.engine.step(s0, g, obs)
        ga = a.fp.grad.clone()
        sb = b.engine.step(s0, g, obs)
        gb = b.fp.grad.clone()
        torch.cuda.synchronize()
        assert torch.isfinite(ga).all()
        assert torch.equal(ga, gb), it
        assert torch.equal(sa.raw[:16], sb.raw[:16]), it
        assert float(sa["T"]) == float(sb["T"])
    assert len(b.engine._bwd_graphs) == 1


def test_backward_graph_statistics_through_the_optimizer_commit(monkeypatch):
    """Under train_step the replayed graph's statistics reach the iteration's row through the
    optimizer's commit launch (no separate copy): rows, skipped flags, gradients and parameters
    equal the eager trainer's, iteration by iteration."""
    monkeypatch.setenv("MACBF_BWD_GRAPH", "0")
    a = _trainer(True, T=20)
    monkeypatch.setenv("MACBF_BWD_GRAPH", "1")
    b = _trainer(True, T=20)
    b.fp.flat.copy_(a.fp.flat)
    b.engine.after_update()
    s0, g, obs = a.sample()
    for it in range(4):
        sa = a.train_step(s0, g, obs)
        sb = b.train_step(s0, g, obs)
        assert sb.flush is not None or it == 0
        assert b.engine._stats_pending is None        # taken by the commit
        torch.cuda.synchronize()
        assert torch.equal(sa.row, sb.row), it
        assert torch.equal(a.fp.flat, b.fp.flat), it
        assert sa["loss_total"] == sb["loss_total"]


def test_backward_graphs_of_several_horizons_replay_exactly(monkeypatch):
    """Early stop changes the horizon T between iterations, so several per-T backward graphs are
    captured into ONE memory pool and replayed in any order. Scenarios of different
    horizons, visited as A B A B A, through the graphed engine give the eager engine's gradient and
    statistics bit for bit, with one graph per horizon."""
    monkeypatch.setenv("MACBF_BWD_GRAPH", "0")
    a = _trainer(True, T=40, B=1, N=32)
    monkeypatch.setenv("MACBF_BWD_GRAPH", "1")
    b = _trainer(True, T=40, B=1, N=32)
    b.fp.flat.copy_(a.fp.flat)
    b.engine.after_update()
    # scenarios with distinct horizons (eager probe runs; the parameters never change: no Adam step)
    scen, horizons = [], set()
    for it in range(40):
        s0, g, obs = a.sample(it)
        T = int(a.engine.rollout(s0, g, obs))
        if T not in horizons:
            horizons.add(T)
            scen.append((s0.clone(), g.clone(), None if obs is None else obs.clone()))
        if len(scen) == 2:
            break
    assert len(scen) == 2, f"no two horizons among the sampled scenarios: {horizons}"
    for it, k in enumerate((0, 1, 0, 1, 0)):
        s0, g, obs = scen[k]
        sa = a.engine.step(s0, g, obs)
        ga = a.fp.grad.clone()
        sb = b.engine.step(s0, g, obs)
        gb = b.fp.grad.clone()
        torch.cuda.synchronize()
        assert torch.isfinite(ga).all()
        assert float(sa["T"]) == float(sb["T"])
        assert torch.equal(ga, gb), (it, k)
        assert torch.equal(sa.raw[:16], sb.raw[:16]), (it, k)
    assert len(b.engine._bwd_graphs) == 2
