"""The native rollout driver (csrc/runtime.cpp) issues the same launches as the Python loop:
identical trajectories, kNN graphs, CBF h slices, horizons and training gradients."""
import pytest
import torch

from macbf_gnn_amd import config as C

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _trainer(acts=False, small=False, **kw):
    """Launch-per-step paths (the persistent small-scene rollout is tested in test_gpu_small.py).
    acts=False: the cooperative node backward recomputes the node MLP (the Python loops always do,
    so the bitwise comparisons below need the recompute on the native path too)."""
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.engine.hip_engine import HipEngine
    from macbf_gnn_amd.parallel import DP
    cfg = C.TrainConfig(num_agents=kw.pop("N", 64), num_envs=kw.pop("B", 4), inner_loops=kw.pop("T", 30),
                        seed=1, device="hip", **kw)
    old = HipEngine.small_rollout
    HipEngine.small_rollout = small
    try:
        tr = Trainer(cfg, device=DEV, dp=DP(device=DEV))
    finally:
        HipEngine.small_rollout = old
    if not acts:
        tr.engine.node_acts = None      # before the drivers are built (lazily, at the first step)
    return tr


def _rollout(tr, native_rollout, s0, g, early_stop):
    eng = tr.engine
    eng.native_rollout = native_rollout
    T = eng.rollout(s0, g, early_stop=early_stop)
    torch.cuda.synchronize()
    BNK = eng.B * eng.N * eng.K
    return (T, eng.S[: T + 1].clone(), eng.idx[:T].clone(), eng.A[:T].clone(), eng.dist[:T].clone(),
            eng.safe[: T + 1].clone(), eng.hbuf[: T * BNK].clone(), eng.hmask[: T * BNK].clone())


@pytest.mark.parametrize("early_stop", [True, False])
def test_native_rollout_matches_python_loop(early_stop):
    tr = _trainer()
    tr.engine.check_every = 1
    s0, g, _ = tr.sample()
    a = _rollout(tr, False, s0, g, early_stop)
    b = _rollout(tr, True, s0, g, early_stop)
    assert a[0] == b[0]
    if early_stop:
        assert a[0] < tr.cfg.inner_loops          # the early stop triggered
    for x, y in zip(a[1:], b[1:]):
        assert torch.equal(x, y)


def test_native_rollout_training_step_matches():
    tr = _trainer(T=12)
    s0, g, _ = tr.sample()
    tr.engine.native_rollout = False
    tr.engine.step(s0, g)
    g_py = tr.fp.grad.clone()
    tr.engine.native_rollout = True
    tr.engine.step(s0, g)
    assert torch.equal(g_py, tr.fp.grad)


def test_bptt_env_groups_match_single_chain():
    """Env groups on separate streams: same gradient up to the slab summation order, and
    deterministic run to run."""
    tr = _trainer(T=10, B=4)
    s0, g, _ = tr.sample()
    tr.engine.step(s0, g)
    g1 = tr.fp.grad.clone()
    from macbf_gnn_amd.engine.hip_engine import HipEngine
    HipEngine.bptt_groups = 2
    try:
        tr2 = _trainer(T=10, B=4)
    finally:
        HipEngine.bptt_groups = 1
    assert tr2.engine.bptt_groups == 2
    tr2.fp.flat.copy_(tr.fp.flat)
    tr2.engine.after_update()
    tr2.engine.step(s0, g)
    g2 = tr2.fp.grad.clone()
    tr2.engine.step(s0, g)
    assert torch.equal(g2, tr2.fp.grad)
    torch.testing.assert_close(g2, g1, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("dim", [2, 3])
def test_native_bptt_matches_python_loop(dim):
    tr = _trainer(T=12, dim=dim)
    s0, g, obs = tr.sample()
    tr.engine.native_bptt = False
    tr.engine.step(s0, g, obs)
    g_py = tr.fp.grad.clone()
    gb_py = tr.engine.Gb.clone()
    tr.engine.native_bptt = True
    tr.engine.step(s0, g, obs)
    assert torch.equal(g_py, tr.fp.grad)
    assert torch.equal(gb_py, tr.engine.Gb)


@pytest.mark.parametrize("dtype,tol", [("fp32", 2e-5), ("bf16", 3e-2), ("fp16", 3e-2)])
def test_node_activations_reuse_matches_recompute(dtype, tol):
    """The cooperative node backward on the node activations the persistent small-scene rollout
    kept (HipEngine.node_acts) against its own recompute: the same gradients up to the forward's
    summation order (the rollout's fragment-layout products vs the backward's row-major ones)."""
    grads = []
    for acts in (True, False):
        tr = _trainer(acts=acts, small=True, T=12, dtype=dtype, N=32, B=2)
        assert (tr.engine.node_acts is not None) == acts
        s0, g, _ = tr.sample()
        tr.engine.step(s0, g)
        torch.cuda.synchronize()
        if acts:
            assert tr.engine._acts_valid
        grads.append(tr.fp.grad.clone())
    a, b = grads
    assert torch.isfinite(a).all()
    err = (a - b).norm() / b.norm()
    assert err < tol, float(err)


@pytest.mark.parametrize("every", [2, 3, 5])
def test_strided_early_stop_check_same_horizon(every):
    """Checking the early-stop criterion every few steps (small scenes) yields the horizon and
    trajectory of a check after every step."""
    tr = _trainer()
    tr.engine.check_every = 1
    s0, g, _ = tr.sample()
    a = _rollout(tr, True, s0, g, True)
    tr2 = _trainer()
    tr2.fp.flat.copy_(tr.fp.flat)
    tr2.engine.after_update()
    tr2.engine.check_every = every
    b = _rollout(tr2, True, s0, g, True)
    assert a[0] == b[0] < tr.cfg.inner_loops
    for x, y in zip(a[1:], b[1:]):
        assert torch.equal(x, y)


def test_device_exploration_noise():
    """Exploration noise (reference train.py:65-67) from the counter-based device RNG: the native
    driver and the Python loop draw the same noise; one coin per (env, step), N(0, scale^2)
    per (agent, axis); deterministic per iteration, fresh across iterations; graph mode runs it."""
    tr = _trainer(T=6, N=256, B=8, add_noise_prob=0.5, noise_scale=0.3)
    s0, g, _ = tr.sample()
    a = _rollout(tr, False, s0, g, False)
    b = _rollout(tr, True, s0, g, False)
    for x, y in zip(a[1:], b[1:]):
        assert torch.equal(x, y)
    # noise-free reference of the same first step: the difference is the noise of step 0
    tr0 = _trainer(T=6, N=256, B=8)
    tr0.fp.flat.copy_(tr.fp.flat)
    tr0.engine.after_update()
    c = _rollout(tr0, True, s0, g, False)
    d = (a[3][0] - c[3][0])                                  # (B, N, D) noise of step 0
    noisy = d.abs().amax(dim=(1, 2)) > 0
    assert 0 < int(noisy.sum()) < 8                          # coin per env (p = 0.5, 8 envs)
    z = d[noisy].flatten() / 0.3
    assert abs(z.mean().item()) < 0.1 and abs(z.std().item() - 1.0) < 0.1
    assert torch.all(d[~noisy] == 0)
    # next iteration: different draws
    tr.step_count += 1
    e = _rollout(tr, True, s0, g, False)
    assert not torch.equal(e[3], b[3])
    tr.step_count -= 1
    f = _rollout(tr, True, s0, g, False)
    assert torch.equal(f[3], b[3])


def test_graph_mode_with_noise_matches_eager():
    tr_e = _trainer(T=8, N=32, B=3, add_noise_prob=1.0, early_stop=False)
    tr_g = _trainer(T=8, N=32, B=3, add_noise_prob=1.0, early_stop=False, graph=True)
    tr_g.fp.flat.copy_(tr_e.fp.flat)
    tr_g.engine.after_update()
    s0, g, _ = tr_e.sample(0)
    tr_e.engine.step(s0, g)
    tr_g.engine.step(s0, g)
    torch.cuda.synchronize()
    torch.testing.assert_close(tr_g.fp.grad, tr_e.fp.grad, rtol=1e-5, atol=1e-7)


def test_rollout_sums_order_independent_at_1024_agents():
    """Per-env goal-distance / action sums of 1024-agent envs (32 waves per env) are fixed-point
    integer atomics: repeated rollouts give bit-identical sums and the same horizon (the early-
    stop input must not depend on the order in which waves finish)."""
    tr = _trainer(N=1024, B=4, T=25)
    tr.engine.check_every = 1
    s0, g, _ = tr.sample()
    runs = [_rollout(tr, True, s0, g, True) for _ in range(3)]
    for r in runs[1:]:
        assert r[0] == runs[0][0]
        for x, y in zip(r[1:], runs[0][1:]):
            assert torch.equal(x, y)
    assert torch.equal(tr.engine.act[: runs[0][0]], tr.engine.act[: runs[0][0]])


def test_published_early_stop_matches_copy_path(monkeypatch):
    """The controller kernels publish the per-env goal-distance sums to host-coherent memory
    (csrc/ctrl.hip publish_step, no per-step queue marker / side-stream copy): over consecutive
    rollouts -- each a new generation, the previous one's late steps still in flight when the
    host breaks -- horizons and trajectories equal the marker + copy path's."""
    monkeypatch.setenv("MACBF_PUBLISH", "0")
    tr_c = _trainer()
    tr_c.engine._driver()                  # the driver reads MACBF_PUBLISH when it is built
    monkeypatch.setenv("MACBF_PUBLISH", "1")
    tr_p = _trainer()
    tr_p.engine._driver()
    tr_p.fp.flat.copy_(tr_c.fp.flat)
    tr_p.engine.after_update()
    for tr in (tr_c, tr_p):
        tr.engine.check_every = 1
    stopped = 0
    for rep in range(5):
        s0, g, _ = tr_c.sample()
        a = _rollout(tr_c, True, s0, g, True)
        b = _rollout(tr_p, True, s0, g, True)
        assert a[0] == b[0]
        stopped += a[0] < tr_c.cfg.inner_loops
        for x, y in zip(a[1:], b[1:]):
            assert torch.equal(x, y)
    assert stopped >= 1

