"""Reference-precision (fp32) HIP path: the 3-term split-bf16 ("x3") kernels against the fp32
oracle with UNROUNDED fp32 weights (MI355X only). Targets: kernel outputs <= 1e-4 relative,
gradients <= 1e-3 relative norm per tensor (the bf16 path is checked against a bf16-operand
emulation at 1e-2 forward / 2e-2 kernel and step gradients in test_gpu_backward.py; reference
precision: /root/reference/core.py:47-48, train.py:167-172).

Per-node state gradients are compared tie-aware (tests/numerics.py ctrl_tie_nodes): an edge whose
relu pre-activation sits within the x3 rounding (~1e-6 of sum |terms|) of zero takes the other relu'
branch than the fp32 oracle (measured: the two outlier edges of the 40-agent CBF case have
pre-activations at 2.3e-7 and 3.1e-7 of sum |terms|, round 2); such a tie moves only the gradient
of that edge's two endpoints. The nodes a float64 tie test flags (relu / radius / max-pool
near-ties within 3e-5 of sum |terms|) are exempt from the 1e-3 bound, every other node is held to
it, and the number of exempt nodes is bounded per case at ~2x its measured count (VERDICT r4
weak #8; round 4 trimmed the worst 2.5 % of nodes instead). Parameter gradients (sums over all
edges) are compared whole."""
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
from numerics import cmp_nodes_tie, ctrl_tie_nodes, edge_ties_to_nodes

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
P32 = "fp32"


def _nets(seed=0, dim=2):
    torch.manual_seed(seed)
    ctrl, cbf = Controller(2 * dim).to(DEV), CBF(2 * dim).to(DEV)
    fp = FlatParams({"controller": ctrl, "cbf": cbf}, device=DEV)
    return ctrl, cbf, fp, PackedWeights(fp, dim, torch.float32)


def _states(lead, N, seed=0, vscale=0.6, dens=1.0):
    g = torch.Generator().manual_seed(seed)
    L_ = math.sqrt(max(1.0, N / 8.0)) * dens
    p = torch.rand(*lead, N, 2, generator=g) * L_
    v = (torch.rand(*lead, N, 2, generator=g) - 0.5) * 2 * vscale
    return torch.cat([p, v], -1).to(DEV)


def _rel(got, ref):
    got, ref = got.double().flatten(), ref.double().flatten()
    rn = ref.norm().item()
    return (got - ref).norm().item() / max(rn, 1e-30)


def _cmp(got, ref, name, rel):
    e = _rel(got, ref)
    assert e <= rel, f"{name}: rel err {e:.3e} > {rel:.0e}"




def _cbf_tie_free(p, S, idx, tau=3e-5):
    """Evaluations whose every CBF relu pre-activation is farther than tau * sum|terms| from 0
    (float64): the split products carry <= ~2^-15 relative error, so the kernel's relu' agrees
    with the oracle's on these; the rest are ties (module docstring)."""
    x, _ = O.cbf_features(S.double(), idx)
    z = x
    ok = torch.ones(x.shape[:-1], dtype=torch.bool, device=x.device)
    for i in (0, 2, 4):
        W = p[f"cbf_net.{i}.weight"].detach().double()
        W = W.reshape(W.shape[0], -1)
        bb = p[f"cbf_net.{i}.bias"].detach().double()
        pre = z @ W.t() + bb
        ok &= ((pre.abs() / (z.abs() @ W.abs().t() + bb.abs())) > tau).all(-1)
        z = torch.relu(pre)
    return ok


def _unpack(fp, maps, reds):
    g = torch.zeros_like(fp.flat)
    offs = {pn: o for (m, pn, shape, o, n) in fp.specs}
    for name, red in reds.items():
        s, d = maps[name](offs)
        g.index_add_(0, torch.as_tensor(d, device=DEV), red.index_select(0, torch.as_tensor(s, device=DEV)))
    return g


def _param_grads(fp, flat_grad, module_name):
    return {pn: flat_grad[o:o + n].view(shape) for m, pn, shape, o, n in fp.specs if m == module_name}


def test_packed_planes_reconstruct_fp32():
    """hi + lo planes of every packed weight reproduce the fp32 master value to ~2^-16."""
    ctrl, cbf, fp, pw = _nets(1)
    torch.cuda.synchronize()
    for buf in (pw.ctrl_w, pw.cbf_w):
        f = buf.view(-1, 2, 512).float()
        full = f[:, 0] + f[:, 1]
        assert torch.all((f[:, 1].abs() <= f[:, 0].abs() * 2 ** -8 + 1e-30))
        assert torch.isfinite(full).all()
    n = pw.cbf_rm.numel() // 2
    rm = pw.cbf_rm.float()
    W2 = cbf.params_dict()["cbf_net.2.weight"].reshape(128, 64)
    img = (rm[:n] + rm[n:])[: 128 * 68].view(128, 68)[:, :64]
    assert (img - W2).abs().max().item() <= 2 ** -16 * W2.abs().max().item()


@pytest.mark.parametrize("B,T,N", [(1, 2, 8), (2, 3, 50), (4, 3, 256)])
def test_cbf_fwd_fp32(B, T, N):
    ctrl, cbf, fp, pw = _nets(1)
    K = min(N, C.TOP_K)
    S = torch.stack([_states((B,), N, seed=10 + t, vscale=1.0) for t in range(T + 1)], 0).contiguous()
    S[..., :2] *= 0.5
    idx = torch.stack([O.knn_idx(S[t], K) for t in range(T)], 0).to(torch.int32).contiguous()
    h = torch.empty(T, B, N, K, device=DEV)
    hn = torch.empty_like(h)
    native.cbf_fwd(S, idx, pw.cbf_w, pw.cbf_off["w1f"], pw.cbf_v, two=True, h_out=h, hn_out=hn, prec=P32)
    torch.cuda.synchronize()
    with torch.no_grad():
        href = O.cbf_forward(cbf.params_dict(), S[:T], idx.long())
        hnref = O.cbf_forward(cbf.params_dict(), S[1:], idx.long())
    _cmp(h, href, "h", 1e-4)
    _cmp(hn, hnref, "h'", 1e-4)
    assert (h - href).abs().max().item() <= 1e-4 * href.abs().max().item()


def test_cbf_hfwd_fp32():
    """Deduplicated forward (row-major W2/W3 images with lo planes) == oracle h at 1e-4: main
    slots on s_t, extras (every 5th slot) on s_{t+1} with their own neighbour slots; radius masks
    exact."""
    ctrl, cbf, fp, pw = _nets(2)
    T, B, N = 3, 2, 96
    K = C.TOP_K
    S = _states((T + 1, B), N, seed=4, dens=0.6).contiguous()
    idx = torch.stack([O.knn_idx(S[t], K) for t in range(T)]).to(torch.int32).contiguous()
    idx1 = torch.stack([O.knn_idx(S[t + 1], K) for t in range(T)]).to(torch.int32).contiguous()
    E = T * B * N * K
    ex = torch.arange(0, E, 5, dtype=torch.int32, device=DEV)
    src = torch.full((2 * E,), -1, dtype=torch.int32, device=DEV)
    src[E:E + ex.numel()] = ex
    nev = torch.tensor([E + ex.numel()], dtype=torch.int32, device=DEV)
    h = torch.zeros(2 * E, device=DEV)
    m = torch.zeros(2 * E, dtype=torch.uint8, device=DEV)
    native.cbf_hfwd(S, idx, idx1, src, nev, pw.cbf_w, pw.cbf_off["w1f"], pw.cbf_rm, pw.cbf_v, h, m, prec=P32)
    torch.cuda.synchronize()
    with torch.no_grad():
        href = O.cbf_forward(cbf.params_dict(), S[:T], idx.long()).reshape(-1)
        h1ref = O.cbf_forward(cbf.params_dict(), S[1:], idx1.long()).reshape(-1)[ex.long()]
        _, mref = O.cbf_features(S[:T], idx.long())
        _, m1ref = O.cbf_features(S[1:], idx1.long())
    _cmp(h[:E], href, "h", 1e-4)
    _cmp(h[E:E + ex.numel()], h1ref, "h' extras", 1e-4)
    assert torch.equal(m[:E].bool(), mref.reshape(-1).bool())
    assert torch.equal(m[E:E + ex.numel()].bool(), m1ref.reshape(-1)[ex.long()].bool())
    assert m[:E].bool().any()


@pytest.mark.parametrize("B,N", [(1, 8), (2, 32), (3, 100), (64, 1024)])
def test_ctrl_fwd_fp32(B, N):
    ctrl, cbf, fp, pw = _nets(3)
    s = _states((B,), N, seed=1)
    g = (s[..., :2] + (torch.rand(B, N, 2, device=DEV) - 0.5)).contiguous()
    K = min(N, C.TOP_K)
    idx = O.knn_idx(s, K).to(torch.int32).contiguous()
    A = torch.empty(B, N, 2, device=DEV)
    Sn = torch.empty(B, N, 4, device=DEV)
    pooled = torch.empty(B, N, 256, dtype=torch.bfloat16, device=DEV)
    am = torch.empty(B, N, 128, dtype=torch.uint8, device=DEV)
    native.ctrl_fwd(s, g, idx, pw.ctrl_w, pw.ctrl_off["ew1f"], pw.ctrl_off["nw1f"], pw.ctrl_v, A, Sn, None, None,
                    pooled=pooled, argmax=am, prec=P32)
    torch.cuda.synchronize()
    with torch.no_grad():
        aref = O.controller_forward(ctrl.params_dict(), s, g, idx.long())
    _cmp(A, aref, "a", 1e-4)
    sn_ref = s + torch.cat([s[..., 2:], A], -1) * C.TIME_STEP
    torch.testing.assert_close(Sn, sn_ref, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("T,B,N", [(2, 1, 16), (3, 2, 40)])
def test_cbf_bwd_fp32(T, B, N):
    ctrl, cbf, fp, pw = _nets(2)
    K = min(N, C.TOP_K)
    S = _states((T + 1, B), N, seed=7, dens=0.6).contiguous()
    idx = torch.stack([O.knn_idx(S[t], K) for t in range(T)]).to(torch.int32).contiguous()
    g = torch.Generator(device="cpu").manual_seed(3)
    dh_raw = torch.randn(2, T, B, N, K, generator=g).to(DEV)
    p = {k: v.detach().clone().requires_grad_(True) for k, v in cbf.params_dict().items()}
    # relu ties (module docstring) get no upstream gradient: ~1 % of the evaluations here
    dh_raw[0] *= _cbf_tie_free(p, S[:T], idx.long())
    dh_raw[1] *= _cbf_tie_free(p, S[1:], idx.long())
    Sx = S.clone().requires_grad_(True)
    h0 = O.cbf_forward(p, Sx[:T], idx.long())
    h1 = O.cbf_forward(p, Sx[1:], idx.long())
    gr = torch.autograd.grad((dh_raw[0] * h0).sum() + (dh_raw[1] * h1).sum(), [Sx] + list(p.values()))
    m0 = O.cbf_features(S[:T], idx.long())[1]
    m1 = O.cbf_features(S[1:], idx.long())[1]
    dh = torch.stack([dh_raw[0] * m0, dh_raw[1] * m1]).contiguous()
    dE = torch.zeros(2, T, B, N, K, 4, device=DEV)
    nb = native.cbf_bwd_grid(2 * T * B * N * K, DEV)
    part = torch.zeros(nb, native.CBF_PARTIAL, device=DEV)
    native.cbf_bwd(S, idx, dh, pw.cbf_w, pw.cbf_off["w1f"], pw.cbf_rm, pw.cbf_v, passes=2, dE=dE, partial=part,
                   num_blocks=nb, prec=P32)
    rptr = torch.zeros(T * B, N + 1, dtype=torch.int32, device=DEV)
    red_e = torch.zeros(T * B, N * K, dtype=torch.int32, device=DEV)
    native.rev_csr(idx.view(T * B, N, K), rptr, red_e)
    dS = torch.zeros(T + 1, B, N, 4, device=DEV)
    native.node_reduce(dE, rptr, red_e, dS, T=T, B=B, N=N, K=K, passes=2)
    red = torch.zeros(native.CBF_PARTIAL, device=DEV)
    native.reduce_rows(part, red)
    torch.cuda.synchronize()
    _cmp(dS, gr[0], "dL/dS", 1e-3)
    mine = _param_grads(fp, _unpack(fp, {"cbf": L.cbf_grad_map}, {"cbf": red}), "cbf")
    for (k, _), ref in zip(p.items(), gr[1:]):
        _cmp(mine[k], ref, k, 1e-3)


def test_fused_cbf_fp32_matches_two_kernel_path():
    ctrl, cbf, fp, pw = _nets(5)
    T, B, N = 3, 2, 96
    K = C.TOP_K
    S = _states((T + 1, B), N, seed=9, dens=0.5).contiguous()
    idx = torch.stack([O.knn_idx(S[t], K) for t in range(T)]).to(torch.int32).contiguous()
    dang = torch.stack([O.ttc_mask_knn(S[t], idx[t].long()) for t in range(T)]).to(torch.uint8).contiguous()
    valid = torch.ones(T, B, dtype=torch.uint8, device=DEV)
    counts = torch.tensor([float(dang.sum()), float((1 - dang).sum()), 0.0], device=DEV)
    E = T * B * N * K
    nbf = native.cbf_fwd_grid(E, DEV)
    pf = torch.zeros(nbf, 10, device=DEV)
    dh = torch.zeros(2, T, B, N, K, device=DEV)
    native.cbf_fwd(S, idx, pw.cbf_w, pw.cbf_off["w1f"], pw.cbf_v, dang=dang, valid=valid, two=True, dh_out=dh,
                   counts=counts, partial=pf, num_blocks=nbf, prec=P32)
    nb = native.cbf_bwd_grid(2 * E, DEV)
    p1 = torch.zeros(nb, native.CBF_PARTIAL, device=DEV)
    dE1 = torch.zeros(2, T, B, N, K, 4, device=DEV)
    native.cbf_bwd(S, idx, dh, pw.cbf_w, pw.cbf_off["w1f"], pw.cbf_rm, pw.cbf_v, passes=2, dE=dE1, partial=p1,
                   num_blocks=nb, prec=P32)
    p2 = torch.zeros(nb, native.CBF_PARTIAL, device=DEV)
    dE2 = torch.zeros(2, T, B, N, K, 4, device=DEV)
    native.cbf_bwd(S, idx, None, pw.cbf_w, pw.cbf_off["w1f"], pw.cbf_rm, pw.cbf_v, passes=2, dE=dE2, partial=p2,
                   num_blocks=nb, fused=True, dang=dang, valid=valid, counts=counts, prec=P32)
    r1 = torch.zeros(native.CBF_PARTIAL, device=DEV)
    r2 = torch.zeros(native.CBF_PARTIAL, device=DEV)
    native.reduce_rows(p1, r1)
    native.reduce_rows(p2, r2)
    torch.cuda.synchronize()
    Lo = native.CBF_P_LOSS
    _cmp(r2[Lo + 2:Lo + 10], pf.double().sum(0)[2:], "loss sums", 1e-4)
    _cmp(dE2, dE1, "dE", 1e-4)
    _cmp(r2[:Lo], r1[:Lo], "dW slab", 1e-4)


# exempt tie nodes (flagged AND outside the row tolerance) per case: measured 0 in every case
# (profiles/r5_numerics/tie_counts.jsonl); one allowed against a toolchain flipping a single tie
STEP_TIE_LIMIT = {(1, 32, None): 1, (2, 64, None): 1, (1, 200, None): 1, (2, 64, 64): 1, (1, 200, 128): 1}


@pytest.mark.parametrize("B,N,chunk", [(1, 32, None), (2, 64, None), (1, 200, None), (2, 64, 64), (1, 200, 128)])
def test_ctrl_step_bwd_fp32(B, N, chunk, monkeypatch):
    """One controller backward step against autograd. 32-agent chunks (the default at these
    sizes) run the cooperative node backward (node_bwd_coop), 64 / 128 the per-wave body."""
    if chunk:
        monkeypatch.setenv("MACBF_NODE_CHUNK", str(chunk))
    ctrl, cbf, fp, pw = _nets(4)
    K = min(N, C.TOP_K)
    s = _states((B,), N, seed=11, dens=0.7).contiguous()
    gg = (s[..., :2] + (torch.rand(B, N, 2, device=DEV) - 0.5)).contiguous()
    idx = O.knn_idx(s, K).to(torch.int32).contiguous()
    Gn = torch.randn(B, N, 4, device=DEV)
    act_coef = 0.37
    A = torch.zeros(B, N, 2, device=DEV)
    pooled = torch.zeros(B, N, 256, dtype=torch.bfloat16, device=DEV)
    am = torch.zeros(B, N, 128, dtype=torch.uint8, device=DEV)
    native.ctrl_fwd(s, gg, idx, pw.ctrl_w, pw.ctrl_off["ew1f"], pw.ctrl_off["nw1f"], pw.ctrl_v, A, None, None, None,
                    pooled=pooled, argmax=am, prec=P32)
    nbn, nbe = native.ctrl_bwd_grids(B * N, DEV)
    pn = torch.zeros(nbn, native.CTRL_NODE_PARTIAL, device=DEV)
    pe = torch.zeros(nbe, native.CTRL_EDGE_PARTIAL, device=DEV)
    dP = torch.zeros(B, N, 256, dtype=torch.bfloat16, device=DEV)
    ego = torch.zeros(B, N, 4, device=DEV)
    dEc = torch.zeros(B, N, K, 4, device=DEV)
    valid = torch.ones(B, dtype=torch.uint8, device=DEV)
    native.ctrl_node_bwd(pooled, s, gg, A, Gn, valid, pw.ctrl_rm, pw.node_rm_off, pw.ctrl_v, act_coef, dP, ego,
                         pn, nbn, prec=P32)
    native.ctrl_edge_bwd(s, idx, am, dP, pw.ctrl_w, pw.ctrl_off["ew1f"], pw.ctrl_off["ew2tn"], dEc, pe, nbe, prec=P32)
    rptr = torch.zeros(B, N + 1, dtype=torch.int32, device=DEV)
    red_e = torch.zeros(B, N * K, dtype=torch.int32, device=DEV)
    native.rev_csr(idx, rptr, red_e)
    Gout = torch.zeros(B, N, 4, device=DEV)
    native.node_combine(torch.zeros(B, N, 4, device=DEV), ego, dEc, rptr, red_e, Gn, Gout, K=K)
    rn = torch.zeros(native.CTRL_NODE_PARTIAL, device=DEV)
    re = torch.zeros(native.CTRL_EDGE_PARTIAL, device=DEV)
    native.reduce_rows(pn, rn)
    native.reduce_rows(pe, re)
    torch.cuda.synchronize()
    p = {k: v.detach().clone().requires_grad_(True) for k, v in ctrl.params_dict().items()}
    sx = s.clone().requires_grad_(True)
    a = O.controller_forward(p, sx, gg, idx.long())
    _cmp(A, a.detach(), "a", 1e-4)
    s_next = sx + torch.cat([sx[..., 2:], a], -1) * C.TIME_STEP
    Lsum = (Gn * s_next).sum() + act_coef * O.action_loss_terms(sx, gg, a).sum()
    gr = torch.autograd.grad(Lsum, [sx] + list(p.values()))
    tie = ctrl_tie_nodes(p, s, gg, idx)
    cmp_nodes_tie(Gout, gr[0], tie, "dL/ds_t", limit=STEP_TIE_LIMIT[(B, N, chunk)])
    mine = _param_grads(fp, _unpack(fp, {"node": L.ctrl_node_grad_map, "edge": L.ctrl_edge_grad_map},
                                    {"node": rn, "edge": re}), "controller")
    for (k, _), ref in zip(p.items(), gr[1:]):
        _cmp(mine[k], ref, k, 1e-3)


def _trainer(**kw):
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.parallel import DP
    cfg = C.TrainConfig(num_agents=kw.pop("N", 32), num_envs=kw.pop("B", 2), inner_loops=kw.pop("T", 5),
                        early_stop=False, seed=0, device="hip", dtype="fp32", **kw)
    return Trainer(cfg, device=DEV, dp=DP(device=DEV))


@pytest.mark.parametrize("bptt,reuse,N,extra", [
    (True, True, 32, {}), (False, True, 32, {}), (True, False, 32, {}), (True, True, 256, {}),
    # SURVEY 4.3 shape list: N <= K (the reference's N <= TOP_K branch, core.py:234-237, D3) and
    # the tile-straddling sizes of the 16-agent edge waves / 16-evaluation CBF records
    (True, True, 1, {}), (True, True, 12, {}), (True, True, 13, {}), (True, True, 17, {}),
    (True, False, 13, {}),
    (True, True, 40, dict(dim=3, num_obstacles=2)), (True, True, 9, dict(dim=3, num_obstacles=1)),
])
def test_full_step_grad_fp32(bptt, reuse, N, extra):
    """One full training step (rollout, losses, BPTT backward) of the fp32 HIP engine (its default
    kernels: 16x16x32 CBF / edge backward where they apply) against autograd through the fp32
    oracle engine: every parameter tensor <= 1e-3 relative norm. Below 32 agents the oracle replays
    the engine's trajectory (states, kNN graphs, max-pool argmax slots): with a few dozen agents a
    single max-pool near-tie -- two neighbours' features within the x3 rounding -- routes one
    feature's gradient to another edge and moves a whole parameter tensor by up to ~3e-3
    (scripts/diag_fullstep.py in the git history, seed-dependent at N = 11, 12, 13 and with either edge kernel)."""
    from macbf_gnn_amd.engine.oracle_engine import OracleEngine
    tr = _trainer(bptt=bptt, reuse_nbr_idx=reuse, N=N, B=3 if N < 32 else 2, **extra)
    s0, g, obs = tr.sample()
    stats = tr.engine.step(s0, g, obs)
    g_hip = tr.fp.grad.clone()
    forced = tr.engine.trajectory(int(float(stats["T"]))) if N < 32 else None
    stats_o = OracleEngine(tr).step(s0, g, obs, forced=forced)
    g_ref = tr.fp.grad.clone()
    worst = []
    for m, pn, shape, o, n in tr.fp.specs:
        worst.append((_rel(g_hip[o:o + n], g_ref[o:o + n]), pn))
    worst.sort(reverse=True)
    assert worst[0][0] <= 1e-3, worst[:4]
    assert abs(float(stats["loss_total"]) - stats_o["loss_total"]) <= 1e-4 * abs(stats_o["loss_total"]) + 1e-6


def test_module_api_fp32_default():
    """models.CBF / models.Controller on the device default to the fp32-accurate kernels."""
    torch.manual_seed(5)
    ctrl, cbf = Controller(4).to(DEV), CBF(4).to(DEV)
    s = _states((2,), 40, seed=2)
    g = (s[..., :2] + 0.3).contiguous().requires_grad_(True)
    K = C.TOP_K
    idx = O.knn_idx(s, K)
    sx = s.clone().requires_grad_(True)
    a = ctrl(sx, g)
    h = cbf(sx)
    wa, wh = torch.randn_like(a), torch.randn_like(h)
    ((a * wa).sum() + (h * wh).sum()).backward()
    pc = {k: v.detach().clone().requires_grad_(True) for k, v in ctrl.params_dict().items()}
    pb = {k: v.detach().clone().requires_grad_(True) for k, v in cbf.params_dict().items()}
    s2 = s.clone().requires_grad_(True)
    g2 = g.detach().clone().requires_grad_(True)
    aref = O.controller_forward(pc, s2, g2, idx)
    href = O.cbf_forward(pb, s2, idx)
    gr = torch.autograd.grad((aref * wa).sum() + (href * wh).sum(), [s2, g2])
    _cmp(a.detach(), aref.detach(), "a", 1e-4)
    _cmp(h.detach(), href.detach(), "h", 1e-4)
    tie = ctrl_tie_nodes(pc, s, g, idx) | edge_ties_to_nodes(~_cbf_tie_free(pb, s, idx), idx, s.shape[-2])
    cmp_nodes_tie(sx.grad, gr[0], tie, "dL/ds", limit=1)
    cmp_nodes_tie(g.grad, gr[1], tie, "dL/dg", limit=1)


def test_training_parity_fp32_vs_oracle():
    """60 training iterations of the fp32 HIP engine and of autograd through the fp32 oracle from
    the same initial weights on the same scenarios (each applies its own gradients): the loss
    curves agree to 1e-3 and the parameters stay within 1e-3 relative distance
    (scripts/parity_run.py: 200 iterations, profiles/r2_parity/)."""
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.engine.oracle_engine import OracleEngine
    from macbf_gnn_amd.parallel import DP

    def make(oracle):
        cfg = C.TrainConfig(num_agents=32, num_envs=8, inner_loops=C.INNER_LOOPS, device="hip", seed=0,
                            dtype="fp32", prefetch_data=False)
        tr = Trainer(cfg, device=DEV, dp=DP(device=DEV))
        if oracle:
            tr.engine = OracleEngine(tr)
        return tr

    hip, orc = make(False), make(True)
    for it in range(60):
        a = float(hip.train_step()["loss_total"])
        b = float(orc.train_step()["loss_total"])
        assert abs(a - b) <= 1e-3 * abs(b), (it, a, b)
    d = float((hip.fp.flat.double() - orc.fp.flat.double()).norm() / orc.fp.flat.double().norm())
    assert d <= 1e-3, d


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("B,N", [(3, 200), (2, 1024), (1, 40)])
def test_ctrl_fwd_dense_rows_bitwise(B, N, prec, monkeypatch):
    """K = 12: the dense-row edge phase (32 agents x 12 slots = 12 tiles, agents straddling tiles,
    used when the agents per wave are a multiple of 8) gives bit-identical actions, next states,
    pooled rows, argmax slots and per-env sums to the 2-agent x 16-slot path (apw = 4)."""
    import os
    ctrl, cbf, fp, _ = _nets(5)
    pw = PackedWeights(fp, dtype=torch.float32 if prec == "fp32" else torch.bfloat16)
    s = _states((B,), N, seed=2, dens=0.8)
    g = (s[..., :2] + (torch.rand(B, N, 2, device=DEV) - 0.5)).contiguous()
    idx = O.knn_idx(s, C.TOP_K).to(torch.int32).contiguous()
    prow = 256 if prec == "fp32" else 128
    out = {}
    for apw in ("32", "8", "4"):
        monkeypatch.setenv("MACBF_CTRL_APW", apw)
        A = torch.full((B, N, 2), 7.0, device=DEV)
        Sn = torch.full((B, N, 4), 7.0, device=DEV)
        pooled = torch.zeros(B, N, prow, dtype=torch.bfloat16, device=DEV)
        am = torch.full((B, N, 128), 77, dtype=torch.uint8, device=DEV)
        ds = torch.zeros(B, dtype=torch.int64, device=DEV)
        acs = torch.zeros(B, dtype=torch.int64, device=DEV)
        native.ctrl_fwd(s, g, idx, pw.ctrl_w, pw.ctrl_off["ew1f"], pw.ctrl_off["nw1f"], pw.ctrl_v, A, Sn, ds, acs,
                        pooled=pooled, argmax=am, prec=prec)
        torch.cuda.synchronize()
        out[apw] = (A, Sn, pooled, am, ds, acs)
    assert os.environ["MACBF_CTRL_APW"] == "4"
    for apw in ("32", "8"):
        for x, y, name in zip(out[apw], out["4"], ("A", "Sn", "pooled", "argmax", "dist", "act")):
            assert torch.equal(x, y), (apw, name)
    assert int((out["4"][3] != 255).sum()) > 0


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_ctrl_fwd_dense_rows_bitwise_3d_obstacles(prec, monkeypatch):
    """The dense-row controller step with 3-D states and obstacle nodes (config #5 layout)."""
    from macbf_gnn_amd import env as E
    from macbf_gnn_amd.ops import graph
    ctrl, cbf, fp, _ = _nets(6, dim=3)
    pw = PackedWeights(fp, 3, torch.float32 if prec == "fp32" else torch.bfloat16)
    B, N = 2, 256
    s, g, obs = E.generate_scenarios(B, N, dim=3, num_obstacles=3, seed=4)
    gen = torch.Generator().manual_seed(4)
    s[..., 3:] = (torch.rand(B, N, 3, generator=gen) - 0.5) * 1.2
    s, g, obs = s.to(DEV), g.to(DEV).contiguous(), obs.to(DEV)
    S = graph.node_records(s, obs)
    idx = O.knn_idx(s, C.TOP_K, O.with_obstacles(s, obs)).to(torch.int32).contiguous()
    prow = 256 if prec == "fp32" else 128
    out = {}
    for apw in ("32", "4"):
        monkeypatch.setenv("MACBF_CTRL_APW", apw)
        A = torch.full((B, N, 3), 7.0, device=DEV)
        Sn = S.clone()
        pooled = torch.zeros(B, N, prow, dtype=torch.bfloat16, device=DEV)
        am = torch.full((B, N, 128), 77, dtype=torch.uint8, device=DEV)
        native.ctrl_fwd(S, g, idx, pw.ctrl_w, pw.ctrl_off["ew1f"], pw.ctrl_off["nw1f"], pw.ctrl_v, A, Sn, None, None,
                        pooled=pooled, argmax=am, prec=prec)
        torch.cuda.synchronize()
        out[apw] = (A, Sn, pooled, am)
    for x, y, name in zip(out["32"], out["4"], ("A", "Sn", "pooled", "argmax")):
        assert torch.equal(x, y), name
