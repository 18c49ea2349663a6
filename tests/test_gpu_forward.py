"""GPU numerics of the forward HIP kernels against the fp32 PyTorch oracle (MI355X only)."""
import math

import numpy as np
import pytest
import torch

from macbf_gnn_amd import config as C
from macbf_gnn_amd import oracle as O
from macbf_gnn_amd.models import CBF, Controller
from macbf_gnn_amd.ops import native
from macbf_gnn_amd.ops.weights import PackedWeights
from macbf_gnn_amd.utils.params import FlatParams

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _states(B, N, seed=0, vscale=0.5):
    g = torch.Generator().manual_seed(seed)
    L = math.sqrt(max(1.0, N / 8.0))
    p = torch.rand(B, N, 2, generator=g) * L
    v = (torch.rand(B, N, 2, generator=g) - 0.5) * 2 * vscale
    s = torch.cat([p, v], -1)
    goals = p + (torch.rand(B, N, 2, generator=g) - 0.5)
    return s.to(DEV), goals.to(DEV)


def _nets(seed=0):
    torch.manual_seed(seed)
    ctrl, cbf = Controller(4).to(DEV), CBF(4).to(DEV)
    fp = FlatParams({"controller": ctrl, "cbf": cbf}, device=DEV)
    return ctrl, cbf, fp, PackedWeights(fp)


@pytest.mark.parametrize("lanes", [4, 8])
@pytest.mark.parametrize("B,N", [(2, 8), (3, 13), (2, 64), (1, 1100)])
def test_scan_knn_ttc_safety(B, N, lanes):
    _scan_vs_oracle(B, N, lanes)


@pytest.mark.parametrize("lanes", [0, 8])
def test_scan_headline_grid(lanes):
    """64 envs x 1024 agents: the 1,024-thread-block scan (lanes=0 picks it at this size) and
    the 8-lane 256-thread layout give the oracle's lists, bits, counts and safety."""
    _scan_vs_oracle(64, 1024, lanes)


def _scan_vs_oracle(B, N, lanes):
    s, _ = _states(B, N, seed=N)
    K = min(N, C.TOP_K)
    idx = torch.empty(B, N, K, dtype=torch.int32, device=DEV)
    dang = torch.empty(B, N, K, dtype=torch.uint8, device=DEV)
    cnt = torch.zeros(B, 2, dtype=torch.float32, device=DEV)
    safe = torch.zeros(B, dtype=torch.float32, device=DEV)
    native.scan(s, idx, dang, cnt, safe, K=K, lanes=lanes)
    torch.cuda.synchronize()
    ref = O.knn_idx(s, K)
    assert torch.equal(idx.long(), ref)
    dref = O.ttc_mask_knn(s, ref)
    assert torch.equal(dang.bool(), dref)
    assert torch.equal(cnt[:, 0], dref.sum((1, 2)).float())
    assert torch.equal(cnt[:, 1], (~dref).sum((1, 2)).float())
    assert torch.equal(safe, O.safe_agent_count(s).float())


@pytest.mark.parametrize("lanes", [4, 8])
@pytest.mark.parametrize("resort", [True, False])
@pytest.mark.parametrize("B,N,steps", [(2, 13, 3), (2, 300, 4), (1, 1100, 3), (1, 4096, 2)])
def test_scan_temporal_bound_is_exact(B, N, steps, resort, lanes):
    """prev_idx (the previous step's kNN) only tightens the culling: kNN, danger bits, counts
    and safety equal the oracle on moving states, step after step. resort=False keeps the
    first step's Hilbert order (stale curve order: looser culling, identical results)."""
    s, _ = _states(B, N, seed=7 + N, vscale=2.0)
    K = min(N, C.TOP_K)
    prev = None
    for step in range(steps):
        idx = torch.empty(B, N, K, dtype=torch.int32, device=DEV)
        dang = torch.empty(B, N, K, dtype=torch.uint8, device=DEV)
        cnt = torch.zeros(B, 2, dtype=torch.float32, device=DEV)
        safe = torch.zeros(B, dtype=torch.float32, device=DEV)
        native.scan(s, idx, dang, cnt, safe, K=K, prev_idx=prev, sort=resort or step == 0, lanes=lanes)
        torch.cuda.synchronize()
        ref = O.knn_idx(s, K)
        assert torch.equal(idx.long(), ref)
        dref = O.ttc_mask_knn(s, ref)
        assert torch.equal(dang.bool(), dref)
        assert torch.equal(cnt[:, 0], dref.sum((1, 2)).float())
        assert torch.equal(safe, O.safe_agent_count(s).float())
        prev = idx
        s = (s + torch.cat([s[..., 2:], torch.zeros_like(s[..., 2:])], -1) * 0.1).contiguous()


@pytest.mark.parametrize("B,N", [(2, 300), (1, 4096)])
def test_scan_ties_and_out_of_domain(B, N):
    """Morton-ordered scan: exact (d2, index) tie-breaks on a lattice with duplicates, agents
    outside the nominal square (clamped cells), result independent of the visit order."""
    s, _ = _states(B, N, seed=5)
    L = math.sqrt(max(1.0, N / 8.0))
    s[..., :2] = torch.round(s[..., :2] * 4) / 4             # lattice -> many equal distances
    s[:, : N // 10, :2] += 1.5 * L                             # far outside the square
    s[:, N // 10: N // 5, :2] -= 0.7 * L
    K = min(N, C.TOP_K)
    idx = torch.empty(B, N, K, dtype=torch.int32, device=DEV)
    dang = torch.empty(B, N, K, dtype=torch.uint8, device=DEV)
    cnt = torch.zeros(B, 2, device=DEV)
    safe = torch.zeros(B, device=DEV)
    native.scan(s.contiguous(), idx, dang, cnt, safe, K=K)
    torch.cuda.synchronize()
    ref = O.knn_idx(s, K)
    assert torch.equal(idx.long(), ref)
    assert torch.equal(dang.bool(), O.ttc_mask_knn(s, ref))
    assert torch.equal(safe, O.safe_agent_count(s).float())


def test_scan_strided_views():
    """Writes into a (B, T, N, K) trajectory buffer through per-step views."""
    B, T, N = 2, 3, 40
    K = 12
    S = torch.zeros(B, T + 1, N, 4, device=DEV)
    for t in range(T + 1):
        S[:, t] = _states(B, N, seed=t)[0]
    idx = torch.full((B, T, N, K), -1, dtype=torch.int32, device=DEV)
    dang = torch.zeros(B, T, N, K, dtype=torch.uint8, device=DEV)
    cnt = torch.zeros(B, T, 2, device=DEV)
    safe = torch.zeros(B, T + 1, device=DEV)
    for t in range(T):
        native.scan(S[:, t], idx[:, t], dang[:, t], cnt[:, t], safe[:, t], K=K)
    torch.cuda.synchronize()
    for t in range(T):
        assert torch.equal(idx[:, t].long(), O.knn_idx(S[:, t], K))
        assert torch.equal(safe[:, t], O.safe_agent_count(S[:, t]).float())


@pytest.mark.parametrize("B,N", [(1, 8), (2, 32), (3, 100), (64, 1024)])
def test_ctrl_fwd_matches_oracle(B, N):
    ctrl, cbf, fp, pw = _nets()
    s, g = _states(B, N, seed=1)
    K = min(N, C.TOP_K)
    idx = O.knn_idx(s, K).to(torch.int32).contiguous()
    A = torch.empty(B, N, 2, device=DEV)
    Sn = torch.empty(B, N, 4, device=DEV)
    dsum = torch.zeros(B, dtype=torch.int64, device=DEV)     # fixed point (native.FX_DIST / FX_ACT)
    asum = torch.zeros(B, dtype=torch.int64, device=DEV)
    native.ctrl_fwd(s, g, idx, pw.ctrl_w, pw.ctrl_off["ew1f"], pw.ctrl_off["nw1f"], pw.ctrl_v, A, Sn, dsum, asum)
    torch.cuda.synchronize()
    with torch.no_grad():
        aref = O.controller_forward(ctrl.params_dict(), s, g, idx.long())
    err = (A - aref).abs().max().item()
    scale = aref.abs().max().item()
    assert err <= 2e-2 * scale + 1e-3, (err, scale)
    # Euler step consistent with the emitted action
    sn_ref = s + torch.cat([s[..., 2:], A], -1) * C.TIME_STEP
    torch.testing.assert_close(Sn, sn_ref, rtol=1e-6, atol=1e-6)
    dsum = (dsum.double() / native.FX_DIST).float()
    asum = (asum.double() / native.FX_ACT).float()
    torch.testing.assert_close(dsum, torch.linalg.norm(Sn[..., :2] - g, dim=-1).sum(-1), rtol=1e-4, atol=1e-4)
    act_ref = O.action_loss_terms(s, g, A).sum(-1)
    torch.testing.assert_close(asum, act_ref, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("B,T,N", [(1, 2, 8), (2, 3, 50), (4, 5, 256)])
def test_cbf_fwd_h_losses_grads(B, T, N):
    ctrl, cbf, fp, pw = _nets(1)
    K = min(N, C.TOP_K)
    # time-major (T+1, B, N, 4)
    S = torch.stack([_states(B, N, seed=10 + t, vscale=1.0)[0] for t in range(T + 1)], 0).contiguous()
    S[..., :2] *= 0.5          # denser -> more dangerous pairs
    idx = torch.stack([O.knn_idx(S[t], K) for t in range(T)], 0).to(torch.int32).contiguous()
    dang = torch.stack([O.ttc_mask_knn(S[t], idx[t].long()) for t in range(T)], 0).to(torch.uint8).contiguous()
    valid = torch.ones(T, B, dtype=torch.uint8, device=DEV)
    valid[-1, 0] = 0
    h = torch.empty(T, B, N, K, device=DEV)
    hn = torch.empty_like(h)
    dh = torch.empty(2, T, B, N, K, device=DEV)
    vb = valid.bool()[..., None, None]
    nd = (dang.bool() & vb).sum().float()
    ns = (~dang.bool() & vb).sum().float()
    counts = torch.stack([nd, ns]).contiguous()
    nb = native.cbf_fwd_grid(B * T * N * K, DEV)
    partial = torch.zeros(nb, 10, device=DEV)
    native.cbf_fwd(S, idx, pw.cbf_w, pw.cbf_off["w1f"], pw.cbf_v, dang=dang, valid=valid, two=True,
                   h_out=h, hn_out=hn, dh_out=dh, counts=counts, partial=partial, num_blocks=nb)
    torch.cuda.synchronize()
    with torch.no_grad():
        href = O.cbf_forward(cbf.params_dict(), S[:T], idx.long())
        hnref = O.cbf_forward(cbf.params_dict(), S[1:], idx.long())
    scale = href.abs().max().item() + 1e-6
    assert (h - href).abs().max().item() <= 2e-2 * scale + 2e-3
    assert (hn - hnref).abs().max().item() <= 2e-2 * scale + 2e-3
    # loss sums from the kernel's own h/hn must equal the oracle formula on the same values
    sums = O.cbf_loss_sums(h, hn, dang.bool(), valid.bool())
    tot = partial.double().sum(0)
    names = ["n_dang", "n_safe", "loss_dang", "loss_safe", "acc_dang", "acc_safe",
             "loss_dang_deriv", "loss_safe_deriv", "acc_dang_deriv", "acc_safe_deriv"]
    for q, n in enumerate(names):
        assert abs(tot[q].item() - sums[n].item()) <= 1e-3 * max(1.0, abs(sums[n].item())), n
    # upstream grads == autograd of the pooled loss w.r.t. h, h'
    hh = h.clone().requires_grad_(True)
    hhn = hn.clone().requires_grad_(True)
    s2 = O.cbf_loss_sums(hh, hhn, dang.bool(), valid.bool())
    s2["n_dang"], s2["n_safe"] = nd, ns
    out = O.finalize_losses(s2, torch.zeros((), device=DEV), 1.0)
    gh, ghn = torch.autograd.grad(out["total"], [hh, hhn])
    m0 = O.cbf_features(S[:T], idx.long())[1]
    m1 = O.cbf_features(S[1:], idx.long())[1]
    torch.testing.assert_close(dh[0], gh * m0, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(dh[1], ghn * m1, rtol=1e-4, atol=1e-6)


def test_scenario_invariants():
    from macbf_gnn_amd.ops import scenario
    for N in (8, 32, 1024):
        S, G, _ = scenario.generate(4, N, seed=3, device=DEV)
        torch.cuda.synchronize()
        L = math.sqrt(max(1.0, N / 8.0))
        p = S[..., :2]
        assert torch.all(S[..., 2:] == 0)
        assert torch.all((p >= 0) & (p <= L))
        d = torch.cdist(p, p, compute_mode="donot_use_mm_for_euclid_dist") + torch.eye(N, device=DEV) * 10
        assert d.min().item() > C.DIST_MIN_THRES
        dg = torch.cdist(G, G, compute_mode="donot_use_mm_for_euclid_dist") + torch.eye(N, device=DEV) * 10
        assert dg.min().item() > C.DIST_MIN_THRES
        assert torch.all((G - p).abs() <= 0.5 + 1e-6)
        assert torch.all(p.norm(dim=-1) > C.DIST_MIN_THRES)
    # deterministic in (seed, iteration)
    a = scenario.generate(2, 64, seed=5, iteration=7, device=DEV)
    b = scenario.generate(2, 64, seed=5, iteration=7, device=DEV)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("dim,nobs", [(2, 0), (3, 2)])
def test_scenario_global_workspace_path_is_bitwise_the_lds_path(dim, nobs):
    """The sampler's global-workspace path (large envs; forced here with lds_free) gives the same
    starts and goals, bit for bit, as the LDS path at 1,024 agents (acceptance does not depend on
    the grid)."""
    from macbf_gnn_amd import env as E
    from macbf_gnn_amd.ops import scenario
    B, N = 4, 1024
    obs = (scenario.obstacles(B, N, dim=dim, num_obstacles=nobs, points=12, seed=9, device=DEV) if nobs else None)
    out = []
    for lds_free in (False, True):
        S = torch.empty(B, N, native.rec_width(dim), device=DEV)
        G = torch.empty(B, N, dim, device=DEV)
        native.scenario(S, G, seed=1234, L=E.side_length(N, dim), obs=obs, lds_free=lds_free)
        out.append((S, G))
    torch.cuda.synchronize()
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
