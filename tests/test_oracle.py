"""CPU golden/property tests of the oracle against the reference semantics.
The reference itself cannot be imported (tensorflow/tkinter imports, crashes), so
its well-defined pieces are re-expressed inline here from the cited lines."""
import math

import numpy as np
import pytest
import torch
from hypothesis import given, settings, strategies as st

import core
from macbf_gnn_amd import config as C
from macbf_gnn_amd import env as E
from macbf_gnn_amd import oracle as O
from macbf_gnn_amd.models import CBF, Controller


def test_state_dict_layout_matches_reference():
    ctrl, cbf = Controller(4), CBF(4)
    cs = {k: tuple(v.shape) for k, v in ctrl.state_dict().items()}
    bs = {k: tuple(v.shape) for k, v in cbf.state_dict().items()}
    assert cs == {
        "controller_centr_net.0.weight": (64, 5, 1), "controller_centr_net.0.bias": (64,),
        "controller_centr_net.2.weight": (128, 64, 1), "controller_centr_net.2.bias": (128,),
        "controller_dec_net.0.weight": (64, 132), "controller_dec_net.0.bias": (64,),
        "controller_dec_net.2.weight": (128, 64), "controller_dec_net.2.bias": (128,),
        "controller_dec_net.4.weight": (64, 128), "controller_dec_net.4.bias": (64,),
        "controller_dec_net.6.weight": (4, 64), "controller_dec_net.6.bias": (4,)}
    assert bs == {
        "cbf_net.0.weight": (64, 6, 1), "cbf_net.0.bias": (64,), "cbf_net.2.weight": (128, 64, 1),
        "cbf_net.2.bias": (128,), "cbf_net.4.weight": (64, 128, 1), "cbf_net.4.bias": (64,),
        "cbf_net.6.weight": (1, 64, 1), "cbf_net.6.bias": (1,)}
    assert sum(p.numel() for p in ctrl.parameters()) == 34052
    assert sum(p.numel() for p in cbf.parameters()) == 17089


def test_config_constants():
    import config as ref_cfg
    assert ref_cfg.TIME_STEP == 0.1 and ref_cfg.TOP_K == 12 and ref_cfg.OBS_RADIUS == 1.0
    assert ref_cfg.TRAIN_STEPS == 70000 and ref_cfg.INNER_LOOPS == 50 and ref_cfg.LEARNING_RATE == 1e-4
    assert ref_cfg.TIME_TO_COLLISION == 2.0 and ref_cfg.TIME_TO_COLLISION_CHECK == 0.1
    assert ref_cfg.DIST_MIN_THRES == ref_cfg.DIST_MIN_CHECK == ref_cfg.DIST_MIN_ENLARGED == 0.07


def test_obstacles_match_reference_formulas():
    c = core.generate_obstacle_circle((1.0, 2.0), 0.5, num=12)
    th = np.linspace(0, 2 * np.pi, 12, endpoint=False)
    np.testing.assert_allclose(c, np.stack([1 + 0.5 * np.cos(th), 2 + 0.5 * np.sin(th)], 1))
    r = core.generate_obstacle_rectangle((0.0, 0.0), (2.0, 1.0), num=12)
    assert r.shape == (12, 2)
    # every point lies on the rectangle boundary
    on_x = np.isclose(np.abs(r[:, 0]), 1.0)
    on_y = np.isclose(np.abs(r[:, 1]), 0.5)
    assert np.all(on_x | on_y)
    n1 = int(12 // 2 * 2.0 / 3.0)
    assert np.sum(np.isclose(r[:, 1], 0.5) & (r[:, 0] < 1.0)) >= n1 - 1


@pytest.mark.parametrize("N", [1, 8, 32, 100])
def test_generate_data_invariants(N):
    rng = np.random.default_rng(N)
    s, g = E.generate_data(N, C.DIST_MIN_THRES, rng)
    assert s.shape == (N, 4) and g.shape == (N, 2) and s.dtype == np.float32
    L = math.sqrt(max(1.0, N / 8.0))
    assert np.all(s[:, 2:] == 0)
    assert np.all((s[:, :2] >= 0) & (s[:, :2] <= L))
    assert np.all(np.abs(g - s[:, :2]) <= 0.5)
    d = np.linalg.norm(s[:, None, :2] - s[None, :, :2], axis=-1) + np.eye(N) * 9
    assert d.min() > C.DIST_MIN_THRES
    dg = np.linalg.norm(g[:, None] - g[None], axis=-1) + np.eye(N) * 9
    assert dg.min() > C.DIST_MIN_THRES
    assert np.all(np.linalg.norm(s[:, :2], axis=1) > C.DIST_MIN_THRES)


def test_dynamics_and_euler():
    s = torch.randn(5, 4)
    a = torch.randn(5, 2)
    d = core.dynamics(s, a)
    torch.testing.assert_close(d, torch.cat([s[:, 2:], a], 1))


def test_remove_distant_agents_always_tuple_self_first():
    for n in (5, 12, 30):
        s = torch.rand(n, 4)
        x = s[:, None] - s[None]
        out, ind = core.remove_distant_agents(x, 12)
        k = min(n, 12)
        assert out.shape == (n, k, 4) and ind.shape == (n * k, 2)
        assert torch.all(ind.view(n, k, 2)[:, 0, 1] == torch.arange(n))   # self at slot 0
        # nearest-first ordering
        d = out[..., :2].norm(dim=-1)
        assert torch.all(d[:, 1:] >= d[:, :-1] - 1e-7)


@settings(max_examples=25, deadline=None)
@given(st.integers(2, 40), st.integers(0, 10_000))
def test_knn_equals_bruteforce(n, seed):
    g = torch.Generator().manual_seed(seed)
    s = torch.rand(2, n, 4, generator=g)
    k = min(n, 12)
    idx = O.knn_idx(s, k)
    d2 = ((s[:, :, None, :2] - s[:, None, :, :2]) ** 2).sum(-1)
    kth = torch.sort(d2, -1).values[..., k - 1:k]
    chosen = torch.gather(d2, 2, idx)
    assert torch.all(chosen <= kth + 1e-7)
    assert torch.all(idx[..., 0] == torch.arange(n))


def _ttc_np_reference(s, r, ttc):
    """core.py:212-231 verbatim semantics (numpy, fp64)."""
    sd = s[:, None] - s[None]
    x, y, vx, vy = [sd[..., q] for q in range(4)]
    eye = np.eye(s.shape[0])
    x = x + eye
    y = y + eye
    alpha = vx ** 2 + vy ** 2
    beta = 2 * (x * vx + y * vy)
    gamma = x ** 2 + y ** 2 - r ** 2
    disc = beta ** 2 - 4 * alpha * gamma
    two = (disc > 0) & (gamma > 0) & (beta < 0)
    lt = (-beta - 2 * alpha * ttc < 0) | ((beta + 2 * alpha * ttc) ** 2 < disc)
    return (gamma < 0) | (two & lt)


def test_ttc_all_pairs_matches_reference_and_closed_form():
    rng = np.random.default_rng(0)
    s = rng.uniform(0, 1, size=(40, 4)).astype(np.float64)
    s[:, 2:] -= 0.5
    ref = _ttc_np_reference(s, C.DIST_MIN_CHECK, C.TIME_TO_COLLISION_CHECK)
    got = core.ttc_dangerous_mask_np(s)[..., 0]
    assert np.array_equal(ref, got)
    o = O.ttc_mask_all_pairs(torch.tensor(s, dtype=torch.float64)).numpy()
    assert np.array_equal(o, ref)
    # closed form: min over t in [0, ttc] of |p + v t| < r   <=>  dangerous (generic positions)
    for i in range(40):
        for j in range(40):
            if i == j:
                continue
            p = s[i, :2] - s[j, :2]
            v = s[i, 2:] - s[j, 2:]
            ts = np.linspace(0, C.TIME_TO_COLLISION_CHECK, 2001)
            dmin = np.min(np.linalg.norm(p[None] + v[None] * ts[:, None], axis=1))
            if abs(dmin - C.DIST_MIN_CHECK) > 1e-4:
                assert ref[i, j] == (dmin < C.DIST_MIN_CHECK)


def test_masked_loss_equals_masked_select_formulation():
    g = torch.Generator().manual_seed(0)
    h = torch.randn(3, 4, 10, 12, generator=g)
    hn = torch.randn(3, 4, 10, 12, generator=g)
    dang = torch.rand(3, 4, 10, 12, generator=g) < 0.3
    valid = torch.ones(3, 4, dtype=torch.bool)
    sums = O.cbf_loss_sums(h, hn, dang, valid)
    hd = torch.masked_select(h, dang)
    hs = torch.masked_select(h, ~dang)
    assert torch.isclose(sums["loss_dang"], torch.relu(hd + 1e-3).sum())
    assert torch.isclose(sums["loss_safe"], torch.relu(-hs).sum())
    assert sums["n_dang"] == hd.numel()
    assert torch.isclose(sums["acc_safe"], (hs > 0).float().sum())


def test_controller_maxpool_grad_reaches_edge_mlp():
    """D13: the reference pooled argmax *indices*, so its edge MLP never got gradient."""
    torch.manual_seed(0)
    ctrl = Controller(4)
    s = torch.rand(1, 20, 4)
    g = torch.rand(1, 20, 2)
    a = ctrl(s, g)
    a.sum().backward()
    assert ctrl.controller_centr_net[0].weight.grad.abs().sum() > 0
    assert ctrl.controller_centr_net[2].weight.grad.abs().sum() > 0


def test_core_api_runs_small_N():
    """D3: N <= TOP_K must work through every core.py entry point."""
    torch.manual_seed(0)
    ctrl, cbf = Controller(4), CBF(4)
    s, g = E.generate_data(8, C.DIST_MIN_THRES, np.random.default_rng(1))
    s = torch.from_numpy(s)
    g = torch.from_numpy(g)
    a = ctrl(s, g)
    assert a.shape == (8, 2)
    h = cbf(s)
    assert h.shape == (8, 1, 8)
    lb = core.loss_barrier(h, s)
    ld = core.loss_derivatives(s, a, h, cbf)
    la = core.loss_actions(s, g, a)
    assert len(lb) == 4 and len(ld) == 4 and la.dim() == 0
    m = core.ttc_dangerous_mask(s)
    assert m.shape == (8, 8, 1) and m.dtype == torch.bool


def test_oracle_bptt_gradient_flows_through_states():
    """Barrier-loss grads reach controller weights through the rollout states (C19)."""
    torch.manual_seed(0)
    ctrl, cbf = Controller(4), CBF(4)
    s0, g = E.generate_batch(1, 16, seed=1)
    traj = O.rollout(ctrl.params_dict(), s0, g, inner_loops=4, early_stop=False)
    T = traj["A"].shape[1]
    h = O.cbf_forward(cbf.params_dict(), traj["S"][:, :T], traj["idx"])
    h.sum().backward()
    assert ctrl.controller_dec_net[0].weight.grad.abs().sum() > 0


def test_oracle_total_loss_gradcheck_fp64():
    """fp64 finite-difference check of the oracle's full BPTT loss: the GPU
    backward kernels are validated against these autograd gradients, so they must be right.
    Hinges / max-pool / kNN are piecewise smooth; the random point is generic."""
    torch.manual_seed(3)
    ctrl, cbf = Controller(4).double(), CBF(4).double()
    s0, g = E.generate_batch(1, 6, seed=7)
    s0, g = s0.double(), g.double()
    s0[..., 2:] = 0.3 * torch.randn_like(s0[..., 2:])
    cp, bp = ctrl.params_dict(), cbf.params_dict()
    # a subset of tensors keeps gradcheck fast; every layer type of both nets is represented
    names_c = ["controller_centr_net.2.bias", "controller_dec_net.4.bias", "controller_dec_net.6.weight"]
    names_b = ["cbf_net.0.bias", "cbf_net.4.bias", "cbf_net.6.weight"]
    leaves = [cp[n].detach().clone().requires_grad_(True) for n in names_c]
    leaves += [bp[n].detach().clone().requires_grad_(True) for n in names_b]
    s_in = s0.clone().requires_grad_(True)

    def total(s_init, *ps):
        c = dict(cp)
        c.update(zip(names_c, ps[:3]))
        b = dict(bp)
        b.update(zip(names_b, ps[3:]))
        traj = O.rollout(c, s_init, g, inner_loops=3, early_stop=False)
        return O.train_losses(c, b, traj, g)[0]["total"]

    assert torch.autograd.gradcheck(total, (s_in, *leaves), eps=1e-6, atol=1e-5, rtol=1e-4)


def test_bf16_emulation_mode():
    """oracle.emulate_bf16: rounds hidden activations / pre-activation gradients like the bf16
    kernels (small, non-zero change vs the fp32 oracle), restores the fp32 oracle on exit."""
    import torch
    from macbf_gnn_amd import oracle as O
    from macbf_gnn_amd.models import CBF, Controller
    torch.manual_seed(0)
    ctrl, cbf = Controller(4), CBF(4)
    s = torch.cat([torch.rand(2, 24, 2) * 3, torch.rand(2, 24, 2) - 0.5], -1)
    g = s[..., :2] + 0.3
    idx = O.knn_idx(s, 12)
    pc = {k: v.detach().clone().requires_grad_(True) for k, v in ctrl.params_dict().items()}
    pb = {k: v.detach().clone().requires_grad_(True) for k, v in cbf.params_dict().items()}

    def run():
        a = O.controller_forward(pc, s, g, idx)
        h = O.cbf_forward(pb, s, idx)
        gr = torch.autograd.grad(a.square().sum() + h.square().sum(), list(pc.values()) + list(pb.values()))
        return a.detach(), h.detach(), gr

    a0, h0, g0 = run()
    with O.emulate_bf16():
        a1, h1, g1 = run()
    a2, h2, g2 = run()
    assert torch.equal(a0, a2) and torch.equal(h0, h2)
    for x, y in ((a1, a0), (h1, h0)):
        e = ((x - y).norm() / y.norm()).item()
        assert 0 < e < 2e-2
    for x, y in zip(g1, g0):
        assert ((x - y).norm() / y.norm()).item() < 5e-2


def test_forced_rollout_replays_own_trajectory():
    """oracle.rollout(forced=own trajectory): same states, same gradient (straight-through
    replay); pool_slots = the true argmax: same action and gradient as the max-pool."""
    import torch
    from macbf_gnn_amd import oracle as O
    from macbf_gnn_amd.models import CBF, Controller
    torch.manual_seed(1)
    ctrl, cbf = Controller(4), CBF(4)
    s0 = torch.cat([torch.rand(2, 20, 2) * 3, torch.zeros(2, 20, 2)], -1)
    g = s0[..., :2] + 0.4
    pc = {k: v.detach().clone().requires_grad_(True) for k, v in ctrl.params_dict().items()}
    pb = {k: v.detach().clone().requires_grad_(True) for k, v in cbf.params_dict().items()}

    def grads(forced=None):
        tr = O.rollout(pc, s0, g, inner_loops=6, early_stop=False, forced=forced)
        losses, _, _ = O.train_losses(pc, pb, tr, g)
        return tr, torch.autograd.grad(losses["total"], list(pc.values()) + list(pb.values()))

    t0, g0 = grads()
    forced = {"S": t0["S"].detach(), "idx": t0["idx"]}
    t1, g1 = grads(forced)
    assert torch.equal(t1["S"], t0["S"].detach())
    for x, y in zip(g1, g0):
        torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-7)
    # pool slots
    idx = O.knn_idx(s0, 12)
    a, aux = O.controller_forward(pc, s0, g, idx, return_aux=True)
    slots = aux["hm"].argmax(dim=-2)
    slots = torch.where(aux["hm"].max(dim=-2).values > 0, slots, torch.full_like(slots, 255))
    assert float(O.pool_slot_gap(aux["hm"], slots)) == 0.0
    a2 = O.controller_forward(pc, s0, g, idx, pool_slots=slots)
    torch.testing.assert_close(a2, a)
    ga = torch.autograd.grad(a.sum(), list(pc.values()))
    gb = torch.autograd.grad(a2.sum(), list(pc.values()))
    for x, y in zip(ga, gb):
        torch.testing.assert_close(x, y)
