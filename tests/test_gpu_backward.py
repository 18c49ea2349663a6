"""GPU numerics of the hand-written backward kernels against PyTorch autograd on the oracle
(MI355X only). The bf16 kernels are compared with the oracle in bf16-emulation mode
(``oracle.emulate_bf16``: weights, hidden activations, pooled features and pre-activation
gradients rounded where the kernels round), per parameter tensor by relative norm error; the
fp32 (x3) kernels with the plain fp32 oracle (tests/test_gpu_fp32.py holds the per-kernel
fp32 cases)."""
import math

import pytest
import torch

from macbf_gnn_amd import config as C
from macbf_gnn_amd import oracle as O
from macbf_gnn_amd.models import CBF, Controller
from macbf_gnn_amd.ops import layout as L
from macbf_gnn_amd.ops import native
from macbf_gnn_amd.ops.weights import PackedWeights
from macbf_gnn_amd.utils.params import FlatParams
from numerics import rel_cmp

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _nets(seed=0):
    """Weights rounded to bf16 so the fp32 oracle evaluates the same function as the MFMA
    kernels; the remaining differences are bf16 activation/delta rounding."""
    torch.manual_seed(seed)
    ctrl, cbf = Controller(4).to(DEV), CBF(4).to(DEV)
    fp = FlatParams({"controller": ctrl, "cbf": cbf}, device=DEV)
    with torch.no_grad():
        fp.flat.copy_(fp.flat.bfloat16().float())
    return ctrl, cbf, fp, PackedWeights(fp)


def _states(lead, N, seed=0, vscale=0.6, dens=1.0):
    g = torch.Generator().manual_seed(seed)
    L_ = math.sqrt(max(1.0, N / 8.0)) * dens
    p = torch.rand(*lead, N, 2, generator=g) * L_
    v = (torch.rand(*lead, N, 2, generator=g) - 0.5) * 2 * vscale
    return torch.cat([p, v], -1).to(DEV)


def _cmp(got, ref, name, rel, cos=None):
    rel_cmp(got, ref, name, rel, cos)


def _unpack(fp, maps, reds):
    g = torch.zeros_like(fp.flat)
    offs = {pn: o for (m, pn, shape, o, n) in fp.specs}
    for name, red in reds.items():
        s, d = maps[name](offs)
        g.index_add_(0, torch.as_tensor(d, device=DEV), red.index_select(0, torch.as_tensor(s, device=DEV)))
    return g


def _param_grads(fp, flat_grad, module_name):
    out = {}
    for m, pn, shape, o, n in fp.specs:
        if m == module_name:
            out[pn] = flat_grad[o:o + n].view(shape)
    return out


@pytest.mark.parametrize("T,B,N", [(2, 1, 16), (3, 2, 40)])
def test_cbf_bwd_matches_autograd(T, B, N):
    ctrl, cbf, fp, pw = _nets(2)
    K = min(N, C.TOP_K)
    S = _states((T + 1, B), N, seed=7, dens=0.6).contiguous()
    idx = torch.stack([O.knn_idx(S[t], K) for t in range(T)]).to(torch.int32).contiguous()
    g = torch.Generator(device="cpu").manual_seed(3)
    dh_raw = torch.randn(2, T, B, N, K, generator=g).to(DEV)
    p = {k: v.detach().clone().requires_grad_(True) for k, v in cbf.params_dict().items()}
    Sx = S.clone().requires_grad_(True)
    with O.emulate_bf16():
        h0 = O.cbf_forward(p, Sx[:T], idx.long())
        h1 = O.cbf_forward(p, Sx[1:], idx.long())
        Lsum = (dh_raw[0] * h0).sum() + (dh_raw[1] * h1).sum()
        gr = torch.autograd.grad(Lsum, [Sx] + list(p.values()))
    m0 = O.cbf_features(S[:T], idx.long())[1]
    m1 = O.cbf_features(S[1:], idx.long())[1]
    dh = torch.stack([dh_raw[0] * m0, dh_raw[1] * m1]).contiguous()
    dE = torch.zeros(2, T, B, N, K, 4, device=DEV)
    nb = native.cbf_bwd_grid(2 * T * B * N * K, DEV)
    part = torch.zeros(nb, native.CBF_PARTIAL, device=DEV)
    native.cbf_bwd(S, idx, dh, pw.cbf_w, pw.cbf_off["w1f"], pw.cbf_rm, pw.cbf_v, passes=2, dE=dE, partial=part, num_blocks=nb)
    rptr = torch.zeros(T * B, N + 1, dtype=torch.int32, device=DEV)
    red_e = torch.zeros(T * B, N * K, dtype=torch.int32, device=DEV)
    native.rev_csr(idx.view(T * B, N, K), rptr, red_e)
    dS = torch.zeros(T + 1, B, N, 4, device=DEV)
    native.node_reduce(dE, rptr, red_e, dS, T=T, B=B, N=N, K=K, passes=2)
    red = torch.zeros(native.CBF_PARTIAL, device=DEV)
    native.reduce_rows(part, red)
    torch.cuda.synchronize()
    _cmp(dS, gr[0], "dL/dS", rel=TOL_KERNEL)
    flat = _unpack(fp, {"cbf": L.cbf_grad_map}, {"cbf": red})
    mine = _param_grads(fp, flat, "cbf")
    for (k, _), ref in zip(p.items(), gr[1:]):
        _cmp(mine[k], ref, k, rel=TOL_KERNEL)


@pytest.mark.parametrize("B,N", [(1, 32), (2, 64), (1, 200)])
def test_ctrl_step_bwd_matches_autograd(B, N):
    ctrl, cbf, fp, pw = _nets(4)
    K = min(N, C.TOP_K)
    s = _states((B,), N, seed=11, dens=0.7).contiguous()
    gg = (s[..., :2] + (torch.rand(B, N, 2, device=DEV) - 0.5)).contiguous()
    idx = O.knn_idx(s, K).to(torch.int32).contiguous()
    Gn = torch.randn(B, N, 4, device=DEV)
    act_coef = 0.37
    # ---- kernels
    A = torch.zeros(B, N, 2, device=DEV)
    Sn = torch.zeros(B, N, 4, device=DEV)
    pooled = torch.zeros(B, N, 128, dtype=torch.bfloat16, device=DEV)
    am = torch.zeros(B, N, 128, dtype=torch.uint8, device=DEV)
    native.ctrl_fwd(s, gg, idx, pw.ctrl_w, pw.ctrl_off["ew1f"], pw.ctrl_off["nw1f"], pw.ctrl_v, A, Sn, None, None,
                    pooled=pooled, argmax=am)
    nbn, nbe = native.ctrl_bwd_grids(B * N, DEV)
    pn = torch.zeros(nbn, native.CTRL_NODE_PARTIAL, device=DEV)
    pe = torch.zeros(nbe, native.CTRL_EDGE_PARTIAL, device=DEV)
    dP = torch.zeros(B, N, 128, dtype=torch.bfloat16, device=DEV)
    ego = torch.zeros(B, N, 4, device=DEV)
    dEc = torch.zeros(B, N, K, 4, device=DEV)
    valid = torch.ones(B, dtype=torch.uint8, device=DEV)
    native.ctrl_node_bwd(pooled, s, gg, A, Gn, valid, pw.ctrl_rm, pw.node_rm_off, pw.ctrl_v, act_coef, dP, ego,
                         pn, nbn)
    native.ctrl_edge_bwd(s, idx, am, dP, pw.ctrl_w, pw.ctrl_off["ew1f"], pw.ctrl_off["ew2tn"], dEc, pe, nbe)
    rptr = torch.zeros(B, N + 1, dtype=torch.int32, device=DEV)
    red_e = torch.zeros(B, N * K, dtype=torch.int32, device=DEV)
    native.rev_csr(idx, rptr, red_e)
    dS0 = torch.zeros(B, N, 4, device=DEV)
    Gout = torch.zeros(B, N, 4, device=DEV)
    native.node_combine(dS0, ego, dEc, rptr, red_e, Gn, Gout, K=K)
    rn = torch.zeros(native.CTRL_NODE_PARTIAL, device=DEV)
    re = torch.zeros(native.CTRL_EDGE_PARTIAL, device=DEV)
    native.reduce_rows(pn, rn)
    native.reduce_rows(pe, re)
    torch.cuda.synchronize()
    # ---- oracle
    p = {k: v.detach().clone().requires_grad_(True) for k, v in ctrl.params_dict().items()}
    sx = s.clone().requires_grad_(True)
    with O.emulate_bf16():
        a = O.controller_forward(p, sx, gg, idx.long())
        s_next = sx + torch.cat([sx[..., 2:], a], -1) * C.TIME_STEP
        Lsum = (Gn * s_next).sum() + act_coef * O.action_loss_terms(sx, gg, a).sum()
        gr = torch.autograd.grad(Lsum, [sx] + list(p.values()))
    _cmp(A, a.detach(), "a", rel=TOL_FWD)
    _cmp(Gout, gr[0], "dL/ds_t", rel=TOL_KERNEL)
    flat = _unpack(fp, {"node": L.ctrl_node_grad_map, "edge": L.ctrl_edge_grad_map}, {"node": rn, "edge": re})
    mine = _param_grads(fp, flat, "controller")
    for (k, _), ref in zip(p.items(), gr[1:]):
        _cmp(mine[k], ref, k, rel=TOL_KERNEL)


# bf16 kernels vs the bf16-emulating oracle (relative norm error per tensor). Calibrated on
# MI355X (profiles/r2_numerics/): measured errors are 3-10x below these bounds.
TOL_FWD = 1e-2
TOL_KERNEL = 2e-2
TOL_STEP = 2e-2


def _round_params(tr):
    """bf16-representable weights: the oracle then evaluates the kernels' function."""
    with torch.no_grad():
        tr.fp.flat.copy_(tr.fp.flat.bfloat16().float())
    tr.engine.after_update()


def _cmp_tensors(tr, g_hip, g_ref, rel):
    for m, pn, shape, o, n in tr.fp.specs:
        _cmp(g_hip[o:o + n], g_ref[o:o + n], f"{m}.{pn}", rel=rel)


def _trainer(device, **kw):
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.parallel import DP
    cfg = C.TrainConfig(num_agents=kw.pop("N", 32), num_envs=kw.pop("B", 2), inner_loops=kw.pop("T", 5),
                        early_stop=False, seed=0, device="hip" if device.type == "cuda" else "cpu", **kw)
    return Trainer(cfg, device=device, dp=DP(device=device))


@pytest.mark.parametrize("prec", ["bf16", "fp32"])
@pytest.mark.parametrize("bptt,reuse,T", [(True, True, 5), (False, True, 5), (True, False, 5), (False, False, 5),
                                          (True, True, 10), (True, False, 10)])
def test_full_step_grad_matches_oracle(bptt, reuse, T, prec):
    """One training step: HIP engine gradient vs autograd through the oracle engine replaying
    the HIP trajectory, per parameter tensor, for BPTT / no-BPTT and h' on the time-t or on the
    recomputed time-(t+1) neighbour slots. bf16: bf16-rounded weights, oracle in bf16-emulation
    mode; fp32: the x3 kernels vs the fp32 oracle. T = 10 takes the split edge->node reduction
    (early steps on the aux stream during the BPTT)."""
    from macbf_gnn_amd.engine.oracle_engine import OracleEngine
    tr = _trainer(DEV, bptt=bptt, reuse_nbr_idx=reuse, T=T, dtype=prec)
    if prec == "bf16":
        _round_params(tr)
    tr.engine.reduce_late = 4 if T >= 8 else 0
    s0, g, _ = tr.sample()
    stats = tr.engine.step(s0, g)
    g_hip = tr.fp.grad.clone()
    with O.emulate_bf16(prec == "bf16"):     # replay the HIP trajectory, graphs and pooling choices
        stats_o = OracleEngine(tr).step(s0, g, forced=tr.engine.trajectory(int(float(stats["T"]))))
    g_ref = tr.fp.grad.clone()
    _cmp_tensors(tr, g_hip, g_ref, TOL_STEP if prec == "bf16" else 1e-3)
    tf = TOL_FWD if prec == "bf16" else 1e-4
    assert abs(float(stats["loss_total"]) - stats_o["loss_total"]) <= tf * abs(stats_o["loss_total"]) + 1e-6


@pytest.mark.parametrize("T", [4, 12])
def test_full_step_deterministic(T):
    tr = _trainer(DEV, N=64, B=3, T=T)
    tr.engine.reduce_late = 4 if T >= 8 else 0
    s0, g, _ = tr.sample()
    tr.engine.step(s0, g)
    g1 = tr.fp.grad.clone()
    tr.engine.step(s0, g)
    assert torch.equal(g1, tr.fp.grad)


def test_train_steps_hip():
    tr = _trainer(DEV, N=64, B=4, T=20)
    tr.cfg.early_stop = True
    before = tr.fp.flat.clone()
    for _ in range(3):
        st = tr.train_step()
    torch.cuda.synchronize()
    assert torch.isfinite(tr.fp.flat).all()
    assert not torch.equal(before, tr.fp.flat)
    assert 1 <= st["T"] <= 20


def test_fused_cbf_train_kernel_matches_two_kernel_path():
    """cbf_bwd(fused=True) == cbf_fwd (losses + dL/dh) followed by cbf_bwd(dh)."""
    ctrl, cbf, fp, pw = _nets(5)
    T, B, N = 3, 2, 96
    K = C.TOP_K
    S = _states((T + 1, B), N, seed=9, dens=0.5).contiguous()
    idx = torch.stack([O.knn_idx(S[t], K) for t in range(T)]).to(torch.int32).contiguous()
    dang = torch.stack([O.ttc_mask_knn(S[t], idx[t].long()) for t in range(T)]).to(torch.uint8).contiguous()
    valid = torch.ones(T, B, dtype=torch.uint8, device=DEV)
    valid[2, 1] = 0
    counts = torch.tensor([float(dang.sum()), float((1 - dang).sum()), 0.0], device=DEV)
    E = T * B * N * K
    # two-kernel reference
    nbf = native.cbf_fwd_grid(E, DEV)
    pf = torch.zeros(nbf, 10, device=DEV)
    dh = torch.zeros(2, T, B, N, K, device=DEV)
    native.cbf_fwd(S, idx, pw.cbf_w, pw.cbf_off["w1f"], pw.cbf_v, dang=dang, valid=valid, two=True, dh_out=dh,
                   counts=counts, partial=pf, num_blocks=nbf)
    nb = native.cbf_bwd_grid(2 * E, DEV)
    p1 = torch.zeros(nb, native.CBF_PARTIAL, device=DEV)
    dE1 = torch.zeros(2, T, B, N, K, 4, device=DEV)
    native.cbf_bwd(S, idx, dh, pw.cbf_w, pw.cbf_off["w1f"], pw.cbf_rm, pw.cbf_v, passes=2, dE=dE1, partial=p1,
                   num_blocks=nb)
    # fused
    p2 = torch.zeros(nb, native.CBF_PARTIAL, device=DEV)
    dE2 = torch.zeros(2, T, B, N, K, 4, device=DEV)
    native.cbf_bwd(S, idx, None, pw.cbf_w, pw.cbf_off["w1f"], pw.cbf_rm, pw.cbf_v, passes=2, dE=dE2, partial=p2,
                   num_blocks=nb, fused=True, dang=dang, valid=valid, counts=counts)
    r1 = torch.zeros(native.CBF_PARTIAL, device=DEV)
    r2 = torch.zeros(native.CBF_PARTIAL, device=DEV)
    native.reduce_rows(p1, r1)
    native.reduce_rows(p2, r2)
    torch.cuda.synchronize()
    L = native.CBF_P_LOSS
    ref_sums = pf.double().sum(0)
    got = r2[L:L + 10].double()
    assert torch.equal(got[[0, 1]], counts[:2].double())             # counts: the global inputs
    _cmp(got[2:], ref_sums[2:], "loss sums", rel=1e-6)      # measured 2e-8 / 0 / 2e-7
    _cmp(dE2, dE1, "dE", rel=1e-6)
    _cmp(r2[:L], r1[:L], "dW slab", rel=1e-5)


def test_prefetched_sampling_is_identical():
    """Side-stream prefetch of the next scenario batch changes timing only, not the data."""
    a = _trainer(DEV, N=64, B=2, T=6)
    b = _trainer(DEV, N=64, B=2, T=6)
    b._side = None                       # synchronous sampling
    for _ in range(3):
        a.train_step()
        b.train_step()
    torch.cuda.synchronize()
    assert torch.equal(a.fp.flat, b.fp.flat)


def test_full_step_4096_agents_matches_oracle():
    """BASELINE config #4 scale (4096 agents / env, LDS neighbour-tile stress) on a short horizon,
    fp32 (x3) kernels vs the fp32 oracle, per parameter tensor."""
    from macbf_gnn_amd.engine.oracle_engine import OracleEngine
    tr = _trainer(DEV, N=4096, B=2, T=3, dtype="fp32")
    s0, g, _ = tr.sample()
    stats = tr.engine.step(s0, g)
    g_hip = tr.fp.grad.clone()
    OracleEngine(tr).step(s0, g, forced=tr.engine.trajectory(int(float(stats["T"]))))
    g_ref = tr.fp.grad.clone()
    _cmp_tensors(tr, g_hip, g_ref, 1e-3)
    assert torch.isfinite(torch.as_tensor(float(stats["loss_total"])))


@pytest.mark.parametrize("G,N,K,Nn", [(3, 40, 12, 40), (2, 1024, 12, 1120), (1, 6000, 12, 6000), (2, 64, 1, 64),
                                       (3, 700, 16, 700), (2, 4096, 12, 4096)])
def test_rev_csr_matches_sorted_reference(G, N, K, Nn):
    """Reverse CSR (incoming non-self edges per target node, sorted by edge id): the register-held
    path (N*K <= 16384: the headline's 1024 x 12 graphs), the LDS insertion-sort path (4096 x 12)
    and the global-memory path (larger graphs) against torch."""
    gen = torch.Generator().manual_seed(G * N)
    idx = torch.randint(0, Nn, (G, N, K), generator=gen, dtype=torch.int32)
    idx[:, :, 0] = torch.arange(N, dtype=torch.int32)          # self at slot 0
    idx = idx.to(DEV)
    rptr = torch.zeros(G, Nn + 1, dtype=torch.int32, device=DEV)
    red = torch.zeros(G, N * K, dtype=torch.int32, device=DEV)
    native.rev_csr(idx, rptr, red, n_nodes=Nn)
    torch.cuda.synchronize()
    for g in range(G):
        flat = idx[g].reshape(-1).long().cpu()
        e = torch.arange(N * K)
        keep = flat != e // K
        tgt, eid = flat[keep], e[keep]
        order = torch.argsort(tgt * (N * K) + eid)
        counts = torch.bincount(tgt, minlength=Nn)
        ptr_ref = torch.cat([torch.zeros(1, dtype=torch.long), torch.cumsum(counts, 0)])
        assert torch.equal(rptr[g].long().cpu(), ptr_ref)
        assert torch.equal(red[g, : int(ptr_ref[-1])].long().cpu(), eid[order])


@pytest.mark.parametrize("bptt", [True, False])
def test_graph_mode_matches_eager(bptt):
    """Captured-graph iteration (Tmax steps, device-side done masks) == eager iteration: same
    gradient (masked steps contribute nothing) and same valid agent-step count."""
    tr_e = _trainer(DEV, N=32, B=3, T=12, bptt=bptt)
    tr_g = _trainer(DEV, N=32, B=3, T=12, bptt=bptt, graph=True)
    tr_e.cfg.early_stop = True
    tr_g.fp.flat.copy_(tr_e.fp.flat)
    tr_g.engine.after_update()
    for it in range(3):
        s0, g, _ = tr_e.sample(it)
        st_e = tr_e.engine.step(s0, g)
        ge = tr_e.fp.grad.clone()
        st_g = tr_g.engine.step(s0, g)
        torch.cuda.synchronize()
        _cmp(tr_g.fp.grad, ge, f"grad it{it}", rel=1e-4, cos=0.99999)
        assert float(st_g["agent_steps"]) == float(st_e["agent_steps"])
        assert abs(float(st_g["loss_total"]) - float(st_e["loss_total"])) <= 1e-4 * abs(float(st_e["loss_total"])) + 1e-6


def test_graph_mode_training_runs():
    tr = _trainer(DEV, N=32, B=2, T=10, graph=True)
    before = tr.fp.flat.clone()
    for _ in range(4):
        st = tr.train_step()
    torch.cuda.synchronize()
    assert torch.isfinite(tr.fp.flat).all() and not torch.equal(before, tr.fp.flat)
    assert 1 <= float(st["T"]) <= 10


@pytest.mark.parametrize("where", ["assemble", "after"])
def test_device_nan_guard_skips_step_without_host_sync(where, monkeypatch):
    """HIP bf16 path: a non-finite reduced gradient is caught on the device (flag -> fused
    Adam), parameters / moments / step counts stay untouched, the skip is counted. assemble: the
    single-process check inside the gradient-assembly launch (a reduced slab entry poisoned);
    after: the separate check that follows a DP all-reduce (the assembled gradient poisoned)."""
    from macbf_gnn_amd.ops import native
    tr = _trainer(DEV, N=32, B=2, T=4)
    tr.engine.bwd_graph = False                    # eager launches (no graph captures the poison)
    assert tr.engine.check_ok is not None          # single process: the fused check
    before = tr.fp.flat.clone()
    m_before = tr.opt.exp_avg.clone()
    real_step = tr.engine.step
    if where == "assemble":
        real_reduce = native.reduce_multi

        def poisoned_reduce(jobs):
            real_reduce(jobs)
            tr.engine.red_all.fill_(float("nan"))
        monkeypatch.setattr(native, "reduce_multi", poisoned_reduce)
        poisoned = real_step
    else:
        tr.engine.check_ok = None                  # the DP path: grad_check after the all-reduce

        def poisoned(s0, g0, obs=None):
            st = real_step(s0, g0, obs)
            tr.fp.grad[5] = float("inf")
            return st

    tr.engine.step = poisoned
    st = tr.train_step()
    torch.cuda.synchronize()
    assert int(st["skipped"]) == 1 and tr.skipped_steps == 1
    assert torch.equal(before, tr.fp.flat) and torch.equal(m_before, tr.opt.exp_avg)
    assert tr.opt.steps == {"controller": 0, "cbf": 0}
    tr.engine.step = real_step
    monkeypatch.undo()
    st = tr.train_step()
    assert int(st["skipped"]) == 0 and tr.skipped_steps == 1
    assert not torch.equal(before, tr.fp.flat)
    assert tr.opt.steps == {"controller": 1, "cbf": 1}


def test_device_adam_matches_torch_adam():
    """Fused Adam with device step counters == torch.optim.Adam (L2 weight decay)."""
    from macbf_gnn_amd.utils.params import FlatAdam
    ctrl, cbf, fp, _ = _nets(3)
    ref = [p.detach().clone().requires_grad_(True) for p in fp._params()]
    opt_ref = torch.optim.Adam(ref, lr=1e-3, weight_decay=1e-2)
    opt = FlatAdam(fp, lr=1e-3, weight_decay=1e-2)
    g = torch.Generator(device="cpu").manual_seed(0)
    for _ in range(5):
        fp.grad.copy_(torch.randn(fp.grad.shape, generator=g).to(DEV))
        off = 0
        for p in ref:
            p.grad = fp.grad[off:off + p.numel()].view_as(p).clone()
            off += p.numel()
        opt_ref.step()
        opt.step()
    got = fp.flat
    want = torch.cat([p.detach().reshape(-1) for p in ref])
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-6)
    assert opt.steps == {"controller": 5, "cbf": 5}
