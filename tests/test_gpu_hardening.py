"""Failure paths of the device-side bookkeeping: a diverged (NaN) agent state, stale
weight-gradient slab rows, and the device-side step commit (no torch glue kernels).

* A NaN agent must never make its env look done (the fixed-point goal-distance terms saturate),
  the reported action loss must be NaN, and the NaN guard must skip the optimizer step.
* Every BPTT path reduces exactly the slab rows it wrote: NaN-filled slabs before a step must not
  reach the gradient (launch-per-step, env-grouped, no-BPTT and the persistent small-scene path).
"""
import math

import pytest
import torch

from macbf_gnn_amd import config as C

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _trainer(**kw):
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.parallel import DP
    cfg = C.TrainConfig(num_agents=kw.pop("N", 64), num_envs=kw.pop("B", 4), inner_loops=kw.pop("T", 12),
                        seed=kw.pop("seed", 1), device="hip", **kw)
    return Trainer(cfg, device=DEV, dp=DP(device=DEV))


@pytest.mark.parametrize("small", [False, True])
def test_nan_agent_env_never_done_and_step_skipped(small):
    from macbf_gnn_amd.engine.hip_engine import HipEngine
    old = HipEngine.small_rollout
    HipEngine.small_rollout = small
    try:
        tr = _trainer(N=32 if small else 64, T=40)
    finally:
        HipEngine.small_rollout = old
    assert tr.engine.small_rollout == small
    s0, g, _ = tr.sample()
    # a reference rollout stops early
    T0 = tr.engine.rollout(s0, g)
    assert T0 < tr.cfg.inner_loops
    s_bad = s0.clone()
    s_bad[1, 3, 2] = float("nan")                  # env 1, agent 3: vx = NaN
    before = tr.fp.flat.clone()
    st = tr.train_step(s_bad, g)
    torch.cuda.synchronize()
    assert st["T"] == tr.cfg.inner_loops, "a diverged env must never look done"
    assert math.isnan(st["loss_action"])
    assert st["skipped"] == 1
    assert torch.equal(before, tr.fp.flat)
    # the next finite step trains normally and the guard is re-armed
    st = tr.train_step(s0, g)
    torch.cuda.synchronize()
    assert st["skipped"] == 0 and not torch.equal(before, tr.fp.flat)
    assert math.isfinite(st["loss_total"])


def _nan_slabs(tr):
    e = tr.engine
    e.part_node.fill_(float("nan"))
    e.part_edge.fill_(float("nan"))
    for b in list(e._part_cbf.values()) + list(e._part_cbf_nb.values()):
        b.fill_(float("nan"))


@pytest.mark.parametrize("mode", ["per_step", "groups", "no_bptt", "small"])
def test_stale_slab_rows_never_reach_the_gradient(mode):
    from macbf_gnn_amd.engine.hip_engine import HipEngine
    old = HipEngine.bptt_groups
    HipEngine.bptt_groups = 2 if mode == "groups" else 1
    try:
        tr = _trainer(N=32 if mode == "small" else 96, B=4, bptt=mode != "no_bptt")
    finally:
        HipEngine.bptt_groups = old
    s0, g, _ = tr.sample()
    tr.engine.step(s0, g)                       # sizes the lazily allocated slabs
    ref = tr.fp.grad.clone()
    assert torch.isfinite(ref).all()
    _nan_slabs(tr)
    tr.engine.step(s0, g)
    assert torch.isfinite(tr.fp.grad).all()
    assert torch.equal(tr.fp.grad, ref)


def test_step_stats_rows_survive_ring_wrap():
    """Statistics rows live in a ring that is replaced (not overwritten) when full: a StepStats
    read long after its step still holds its own values."""
    from macbf_gnn_amd.engine import hip_engine
    old = hip_engine.STATS_RING
    hip_engine.STATS_RING = 3
    try:
        tr = _trainer(N=32, B=2, T=6)
    finally:
        hip_engine.STATS_RING = old
    stats = [tr.train_step() for _ in range(8)]
    torch.cuda.synchronize()
    raws = [s.raw for s in stats]
    assert len({r.data_ptr() for r in raws}) == 8
    for s in stats:
        assert s["agent_steps"] > 0 and s["skipped"] == 0
