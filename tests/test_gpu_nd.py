"""3-D double integrator + static obstacles (BASELINE config #5) on the HIP kernels vs the
oracle: scan, scenario sampler, reference-module API and the full training step (fp32 kernels
vs the fp32 oracle; bf16 kernels vs the oracle in bf16-emulation mode)."""
import math

import pytest
import torch

from macbf_gnn_amd import config as C
from macbf_gnn_amd import env as E
from macbf_gnn_amd import oracle as O
from macbf_gnn_amd.models import CBF, Controller
from macbf_gnn_amd.ops import graph, native, scenario
from numerics import ctrl_pool_slots, rel_cmp

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _cmp(got, ref, name, rel):
    rel_cmp(got, ref, name, rel)


# (forward, gradient) relative-norm bounds per precision; bf16 against the emulating oracle
TOL = {"fp32": (1e-4, 1e-3), "bf16": (1e-2, 2e-2)}
# the kernels' argmax slots are maxima up to near-ties of this relative size
SLOT_GAP = {"fp32": 1e-5, "bf16": 1e-4}


def _scene(B, N, dim, nobs, seed):
    s, g, obs = E.generate_scenarios(B, N, dim=dim, num_obstacles=nobs, seed=seed)
    gen = torch.Generator().manual_seed(seed)
    s[..., dim:] = (torch.rand(B, N, dim, generator=gen) - 0.5) * 1.2
    return s.to(DEV), g.to(DEV), (obs.to(DEV) if obs is not None else None)


@pytest.mark.parametrize("dim,nobs,N", [(3, 0, 200), (2, 3, 150), (3, 4, 300)])
def test_scan_nd_obstacles(dim, nobs, N):
    s, g, obs = _scene(2, N, dim, nobs, seed=N)
    K = C.TOP_K
    S = graph.node_records(s, obs)
    idx = torch.empty(2, N, K, dtype=torch.int32, device=DEV)
    dang = torch.empty(2, N, K, dtype=torch.uint8, device=DEV)
    cnt = torch.zeros(2, 2, device=DEV)
    safe = torch.zeros(2, device=DEV)
    native.scan(S, idx, dang, cnt, safe, K=K, n_agents=N)
    torch.cuda.synchronize()
    nodes = O.with_obstacles(s, obs)
    ref = O.knn_idx(s, K, nodes)
    assert torch.equal(idx.long(), ref)
    dref = O.ttc_mask_knn(s, ref, nodes)
    assert torch.equal(dang.bool(), dref)
    assert torch.equal(safe, O.safe_agent_count(s, nodes).float())


@pytest.mark.parametrize("nobs,lattice", [(8, False), (0, True)])
def test_scan_3d_temporal_bound_large(nobs, lattice):
    """Config #5 env size (1,024 agents; at B = 3 the launcher picks the 256-thread, 8-lane
    layout -- the production 512-thread config #5 plan is pinned in test_gpu_scan_plans.py) with
    the previous step's kNN as the temporal bound, step after step on moving states: lists, danger bits, counts and safety equal
    the oracle (the path that searches the 3-D cell grid when SCAN_CELL3 is on, the chunk culling
    otherwise). lattice: positions on a coarse grid, many equal distances (exact tie order)."""
    B, N, K = 3, 1024, C.TOP_K
    s, g, obs = _scene(B, N, 3, nobs, seed=11 + nobs)
    if lattice:
        s[..., :3] = torch.round(s[..., :3] * 2) / 2
    prev = None
    for step in range(3):
        S = graph.node_records(s, obs)
        idx = torch.empty(B, N, K, dtype=torch.int32, device=DEV)
        dang = torch.empty(B, N, K, dtype=torch.uint8, device=DEV)
        cnt = torch.zeros(B, 2, device=DEV)
        safe = torch.zeros(B, device=DEV)
        native.scan(S, idx, dang, cnt, safe, K=K, n_agents=N, prev_idx=prev)
        torch.cuda.synchronize()
        nodes = O.with_obstacles(s, obs)
        ref = O.knn_idx(s, K, nodes)
        assert torch.equal(idx.long(), ref), step
        dref = O.ttc_mask_knn(s, ref, nodes)
        assert torch.equal(dang.bool(), dref), step
        assert torch.equal(cnt[:, 0], dref.sum((1, 2)).float()), step
        assert torch.equal(safe, O.safe_agent_count(s, nodes).float()), step
        prev = idx
        s = (s + torch.cat([s[..., 3:], torch.zeros_like(s[..., 3:])], -1) * 0.1).contiguous()


def test_scenario_sampler_3d_obstacles():
    s, g, obs = scenario.generate(3, 256, seed=4, device=DEV, dim=3, num_obstacles=5)
    assert s.shape == (3, 256, 6) and g.shape == (3, 256, 3) and obs.shape == (3, 60, 3)
    for b in range(3):
        p = s[b, :, :3]
        assert torch.all(s[b, :, 3:] == 0)
        d = torch.cdist(p, p, compute_mode="donot_use_mm_for_euclid_dist") + torch.eye(256, device=DEV) * 9
        assert d.min() > C.DIST_MIN_THRES
        assert torch.cdist(p, obs[b], compute_mode="donot_use_mm_for_euclid_dist").min() > C.DIST_MIN_THRES
        assert torch.cdist(g[b], obs[b], compute_mode="donot_use_mm_for_euclid_dist").min() > C.DIST_MIN_THRES
        assert torch.all((g[b] - p).abs() <= C.GOAL_SPREAD + 1e-6)
        L = E.side_length(256, 3)
        assert torch.all((p >= 0) & (p <= L))


def _round_bf16(m):
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(p.bfloat16().float())
    return m


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("dim,nobs", [(3, 0), (3, 2), (2, 2)])
def test_modules_nd_obstacles(dim, nobs, prec):
    torch.manual_seed(dim + nobs)
    ctrl, cbf = Controller(2 * dim).to(DEV), CBF(2 * dim).to(DEV)
    if prec == "bf16":
        ctrl.mfma_dtype = cbf.mfma_dtype = torch.bfloat16
        _round_bf16(ctrl)
        _round_bf16(cbf)
    tf, tg = TOL[prec]
    emu = O.emulate_bf16(prec == "bf16")
    s, g, obs = _scene(2, 64, dim, nobs, seed=9)
    nodes = O.with_obstacles(s, obs)
    K = C.TOP_K
    idx = O.knn_idx(s, K, nodes)
    # CBF
    sx = s.clone().requires_grad_(True)
    h = cbf(sx, obstacles=obs)
    w = torch.randn_like(h)
    (h * w).sum().backward()
    p = {k: v.detach().clone().requires_grad_(True) for k, v in cbf.params_dict().items()}
    s2 = s.clone().requires_grad_(True)
    with emu:
        href = O.cbf_forward(p, s2, idx, nodes=O.with_obstacles(s2, obs))
        gr = torch.autograd.grad((href * w).sum(), [s2] + list(p.values()))
    _cmp(h, href, "h", rel=tf)
    _cmp(sx.grad, gr[0], "cbf dL/ds", rel=tg)
    for (k, prm), ref in zip(cbf.named_parameters(), gr[1:]):
        _cmp(prm.grad, ref, k, rel=tg)
    # controller
    sx = s.clone().requires_grad_(True)
    a = ctrl(sx, g, obstacles=obs)
    wa = torch.randn_like(a)
    (a * wa).sum().backward()
    p = {k: v.detach().clone().requires_grad_(True) for k, v in ctrl.params_dict().items()}
    s2 = s.clone().requires_grad_(True)
    slots, pvals = ctrl_pool_slots(ctrl, s, g, idx, obs)
    with emu:
        aref, aux = O.controller_forward(p, s2, g, idx, nodes=O.with_obstacles(s2, obs), return_aux=True,
                                         pool_slots=slots, pool_values=pvals)
        gr = torch.autograd.grad((aref * wa).sum(), [s2] + list(p.values()))
    assert O.pool_slot_gap(aux["hm"].detach(), slots) < SLOT_GAP[prec]
    with O.emulate_bf16(prec == "bf16"):       # forward checks: the oracle's own max-pool
        afree, aux_f = O.controller_forward(p, s, g, idx, nodes=O.with_obstacles(s, obs), return_aux=True)
    _cmp(pvals, aux_f["pooled"], "pooled", rel=tf)
    _cmp(a, afree, "a", rel=tf)
    _cmp(sx.grad, gr[0], "ctrl dL/ds", rel=tg)
    for (k, prm), ref in zip(ctrl.named_parameters(), gr[1:]):
        _cmp(prm.grad, ref, k, rel=tg)


@pytest.mark.parametrize("dim,nobs,bptt,prec", [(3, 0, True, "fp32"), (3, 3, True, "fp32"), (2, 3, True, "bf16"),
                                                (3, 3, False, "bf16"), (3, 3, True, "bf16")])
def test_full_step_nd_obstacles_matches_oracle(dim, nobs, bptt, prec):
    """One training step, per parameter tensor: fp32 kernels vs the fp32 oracle, bf16 kernels
    (bf16 weights) vs the oracle in bf16-emulation mode."""
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.engine.oracle_engine import OracleEngine
    from macbf_gnn_amd.parallel import DP
    cfg = C.TrainConfig(num_agents=48, num_envs=2, inner_loops=5, early_stop=False, seed=0, device="hip",
                        dim=dim, num_obstacles=nobs, bptt=bptt, dtype=prec)
    tr = Trainer(cfg, device=DEV, dp=DP(device=DEV))
    if prec == "bf16":
        with torch.no_grad():
            tr.fp.flat.copy_(tr.fp.flat.bfloat16().float())
        tr.engine.after_update()
    tf, tg = TOL[prec]
    s0, g, obs = tr.sample()
    stats = tr.engine.step(s0, g, obs)
    g_hip = tr.fp.grad.clone()
    with O.emulate_bf16(prec == "bf16"):     # replay the HIP trajectory, graphs and pooling choices
        stats_o = OracleEngine(tr).step(s0, g, obs, forced=tr.engine.trajectory(int(float(stats["T"]))))
    g_ref = tr.fp.grad.clone()
    for m, pn, shape, o, n in tr.fp.specs:
        _cmp(g_hip[o:o + n], g_ref[o:o + n], f"{m}.{pn}", rel=tg)
    assert abs(float(stats["loss_total"]) - stats_o["loss_total"]) <= tf * abs(stats_o["loss_total"]) + 1e-6
    assert abs(float(stats["safe_agents"]) - stats_o["safe_agents"]) <= 1e-3 * max(1.0, stats_o["safe_agents"])


def test_train_steps_3d_obstacles():
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.parallel import DP
    cfg = C.TrainConfig(num_agents=128, num_envs=4, inner_loops=10, seed=1, device="hip", dim=3,
                        num_obstacles=4)
    tr = Trainer(cfg, device=DEV, dp=DP(device=DEV))
    before = tr.fp.flat.clone()
    for _ in range(3):
        st = tr.train_step()
    torch.cuda.synchronize()
    assert torch.isfinite(tr.fp.flat).all() and not torch.equal(before, tr.fp.flat)
    assert 0.0 <= float(st["safe_agents"]) <= float(st["agent_steps"])


@pytest.mark.parametrize("dim,nobs,N", [(2, 0, 1024), (3, 4, 300), (2, 2, 500)])
def test_device_sampler_matches_host_runtime(dim, nobs, N):
    """The HIP sampler and the C++ host runtime run the same parallel RSA: bit-identical."""
    kw = dict(seed=3, iteration=2, rank=1, dim=dim, num_obstacles=nobs)
    s, g, obs = scenario.generate(4, N, device=DEV, **kw)
    s2, g2, obs2 = scenario.generate(4, N, device="cpu", **kw)
    assert torch.equal(s.cpu(), s2) and torch.equal(g.cpu(), g2)
    if nobs:
        assert torch.equal(obs.cpu(), obs2)
