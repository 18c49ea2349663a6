"""Envs above the 4,096-node LDS staging limit stay on the GPU (VERDICT r1 missing item 4): the
scan stages each env once per step in global memory (boxes in LDS), the scenario sampler keeps
its arrays in a global workspace, the reverse CSR uses its global path. Reference: any N at
/root/reference/core.py:234-250 and controller.py:105-107 (dense pairwise)."""
import math

import pytest
import torch

from macbf_gnn_amd import config as C
from macbf_gnn_amd import oracle as O
from macbf_gnn_amd.ops import native, scenario

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _states(B, N, seed=0, vscale=0.5, dim=2):
    g = torch.Generator().manual_seed(seed)
    L = max(1.0, N / 8.0) ** (1.0 / dim)
    p = torch.rand(B, N, dim, generator=g) * L
    v = (torch.rand(B, N, dim, generator=g) - 0.5) * 2 * vscale
    return torch.cat([p, v], -1).to(DEV)


@pytest.mark.parametrize("B,N,steps", [(2, 8192, 2), (1, 16384, 2)])
def test_scan_global_staging_exact(B, N, steps):
    """kNN (with the temporal bound), danger bits, counts and all-pairs safety at 8K / 16K agents
    equal the oracle bit for bit, over moving states."""
    s = _states(B, N, seed=N, vscale=1.5)
    K = C.TOP_K
    prev = None
    for step in range(steps):
        idx = torch.empty(B, N, K, dtype=torch.int32, device=DEV)
        dang = torch.empty(B, N, K, dtype=torch.uint8, device=DEV)
        cnt = torch.zeros(B, 2, device=DEV)
        safe = torch.zeros(B, device=DEV)
        native.scan(s, idx, dang, cnt, safe, K=K, prev_idx=prev)
        torch.cuda.synchronize()
        ref = O.knn_idx(s, K)
        assert torch.equal(idx.long(), ref)
        dref = O.ttc_mask_knn(s, ref)
        assert torch.equal(dang.bool(), dref)
        assert torch.equal(cnt[:, 0], dref.sum((1, 2)).float())
        assert torch.equal(safe, O.safe_agent_count(s).float())
        prev = idx
        s = (s + torch.cat([s[..., 2:], torch.zeros_like(s[..., 2:])], -1) * 0.1).contiguous()


def test_scan_global_staging_3d():
    s = _states(1, 6000, seed=3, dim=3)
    W = native.rec_width(3)
    S = native.to_records(s)
    K = C.TOP_K
    idx = torch.empty(1, 6000, K, dtype=torch.int32, device=DEV)
    dang = torch.empty(1, 6000, K, dtype=torch.uint8, device=DEV)
    cnt = torch.zeros(1, 2, device=DEV)
    safe = torch.zeros(1, device=DEV)
    assert S.shape[-1] == W
    native.scan(S, idx, dang, cnt, safe, K=K)
    torch.cuda.synchronize()
    ref = O.knn_idx(s, K)
    assert torch.equal(idx.long(), ref)
    assert torch.equal(dang.bool(), O.ttc_mask_knn(s, ref))
    assert torch.equal(safe, O.safe_agent_count(s).float())


@pytest.mark.parametrize("N", [8192, 16384])
def test_sampler_global_workspace_matches_host(N):
    """Device sampler with the global workspace == the C++ host runtime, bit for bit, and the
    scenario invariants hold."""
    kw = dict(seed=4, iteration=1, rank=0)
    s, g, _ = scenario.generate(2, N, device=DEV, **kw)
    s2, g2, _ = scenario.generate(2, N, device="cpu", **kw)
    assert torch.equal(s.cpu(), s2) and torch.equal(g.cpu(), g2)
    p = s[..., :2]
    assert torch.all(s[..., 2:] == 0)
    L = math.sqrt(N / 8.0)
    assert torch.all((p >= 0) & (p <= L))
    assert torch.all((g - p).abs() <= 0.5 + 1e-6)
    idx = O.knn_idx(s, 2)                      # nearest non-self neighbour distance > r
    d = (p - p.gather(1, idx[..., 1:2].expand(-1, -1, 2))).norm(dim=-1)
    assert d.min().item() > C.DIST_MIN_THRES


@pytest.mark.parametrize("N,B,T", [(8192, 1, 2)])
def test_full_step_large_env_matches_oracle(N, B, T):
    """One fp32 training step at 8,192 agents per env (device sampler, global scan staging,
    global reverse CSR) against autograd through the fp32 oracle: every parameter tensor <= 1e-3."""
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.engine.oracle_engine import OracleEngine
    from macbf_gnn_amd.parallel import DP
    cfg = C.TrainConfig(num_agents=N, num_envs=B, inner_loops=T, early_stop=False, seed=0, device="hip",
                        dtype="fp32")
    tr = Trainer(cfg, device=DEV, dp=DP(device=DEV))
    s0, g, _ = tr.sample()
    stats = tr.engine.step(s0, g)
    g_hip = tr.fp.grad.clone()
    OracleEngine(tr).step(s0, g)
    g_ref = tr.fp.grad.clone()
    worst = 0.0
    for m, pn, shape, o, n in tr.fp.specs:
        a, b = g_hip[o:o + n].double(), g_ref[o:o + n].double()
        worst = max(worst, (a - b).norm().item() / max(b.norm().item(), 1e-30))
    assert worst <= 1e-3, worst
    assert math.isfinite(float(stats["loss_total"]))


def test_training_runs_16384_agents():
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.parallel import DP
    cfg = C.TrainConfig(num_agents=16384, num_envs=2, inner_loops=6, seed=1, device="hip", dtype="fp32")
    tr = Trainer(cfg, device=DEV, dp=DP(device=DEV))
    before = tr.fp.flat.clone()
    for _ in range(2):
        st = tr.train_step()
    torch.cuda.synchronize()
    assert torch.isfinite(tr.fp.flat).all() and not torch.equal(before, tr.fp.flat)
    assert float(st["agent_steps"]) > 0


def test_sampler_global_workspace_many_rounds():
    """Repeated large-env sampling (the global-workspace path re-links its cell lists every
    round): every call terminates and equals the host runtime. Regression test for stale L1
    lines of the cell heads, which could link a round's list into the previous one's (a cycle
    the cell walk never left)."""
    for it in range(12):
        kw = dict(seed=100 + it, iteration=it, rank=0)
        s, g, _ = scenario.generate(2, 8192, device=DEV, **kw)
        torch.cuda.synchronize()
        s2, g2, _ = scenario.generate(2, 8192, device="cpu", **kw)
        assert torch.equal(s.cpu(), s2) and torch.equal(g.cpu(), g2)


def test_sampler_concurrent_streams():
    """The trainer samples iteration k+1 on a side stream while iteration k's sampling may still
    run on the main stream: the large-env samplers must not share scratch (regression test: a
    shared global workspace corrupted both cell lists and could hang the walk)."""
    side = torch.cuda.Stream(device=DEV)
    for it in range(4):
        ka = dict(seed=7, iteration=2 * it, rank=0)
        kb = dict(seed=7, iteration=2 * it + 1, rank=0)
        sa, ga, _ = scenario.generate(2, 8192, device=DEV, **ka)
        with torch.cuda.stream(side):
            sb, gb, _ = scenario.generate(2, 8192, device=DEV, **kb)
        torch.cuda.synchronize()
        for (s, g), kw in (((sa, ga), ka), ((sb, gb), kb)):
            s2, g2, _ = scenario.generate(2, 8192, device="cpu", **kw)
            assert torch.equal(s.cpu(), s2) and torch.equal(g.cpu(), g2)


def _knn_chunked(s, K, rows=2048):
    """Oracle kNN of every agent of a (1, N, W) state, computed in query-row chunks (the dense
    N x N distance matrix of 65 K agents would not fit one sort)."""
    out = []
    for q0 in range(0, s.shape[1], rows):
        out.append(O.knn_idx(s[:, q0:q0 + rows], K, nodes=s))
    return torch.cat(out, 1)


def test_scan_global_boxes_65536_agents():
    """envs whose culling boxes exceed LDS (> ~36 K nodes) stay on the GPU --
    the scan reads the boxes from the global workspace. kNN lists, danger bits and counts at
    65,536 agents equal the oracle bit for bit (safety: the all-pairs oracle is O(N^2) memory and
    is covered at 8 K / 16 K above)."""
    N, K = 65536, C.TOP_K
    s = _states(1, N, seed=65, vscale=1.0)
    idx = torch.empty(1, N, K, dtype=torch.int32, device=DEV)
    dang = torch.empty(1, N, K, dtype=torch.uint8, device=DEV)
    cnt = torch.zeros(1, 2, device=DEV)
    safe = torch.zeros(1, device=DEV)
    native.scan(s, idx, dang, cnt, safe, K=K)
    torch.cuda.synchronize()
    ref = _knn_chunked(s, K)
    assert torch.equal(idx.long(), ref)
    dref = O.ttc_mask_knn(s, ref)
    assert torch.equal(dang.bool(), dref)
    assert torch.equal(cnt[:, 0], dref.sum((1, 2)).float())


@pytest.mark.parametrize("N", [20000, 65536])
def test_rev_csr_global_path(N):
    """Reverse CSR of envs whose counters exceed LDS (csrc/graph.hip rev_csr_glb_kernel) against
    a stable sort of the edges by target: same offsets, same edge order."""
    G, K = 2, C.TOP_K
    g = torch.Generator(device=DEV).manual_seed(N)
    idx = torch.randint(0, N, (G, N, K), generator=g, device=DEV, dtype=torch.int32)
    idx[:, :, 0] = torch.arange(N, device=DEV, dtype=torch.int32)     # self slot
    rptr = torch.empty(G, N + 1, dtype=torch.int32, device=DEV)
    red = torch.full((G, N * K), -1, dtype=torch.int32, device=DEV)
    native.rev_csr(idx, rptr, red)
    torch.cuda.synchronize()
    e = torch.arange(N * K, device=DEV)
    for b in range(G):
        j = idx[b].reshape(-1).long()
        keep = j != e // K
        tgt, ed = j[keep], e[keep]
        order = torch.sort(tgt, stable=True).indices
        want = ed[order].to(torch.int32)
        counts = torch.bincount(tgt, minlength=N)
        want_ptr = torch.cat([torch.zeros(1, device=DEV, dtype=torch.long), counts.cumsum(0)]).to(torch.int32)
        assert torch.equal(rptr[b], want_ptr)
        assert torch.equal(red[b, : want.numel()], want)


def test_training_runs_40000_agents():
    """A training iteration at 40,000 agents per env: global scan boxes, global reverse CSR,
    global-workspace sampler."""
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.parallel import DP
    cfg = C.TrainConfig(num_agents=40000, num_envs=1, inner_loops=4, seed=2, device="hip", dtype="fp32")
    tr = Trainer(cfg, device=DEV, dp=DP(device=DEV))
    before = tr.fp.flat.clone()
    st = tr.train_step()
    torch.cuda.synchronize()
    assert torch.isfinite(tr.fp.flat).all() and not torch.equal(before, tr.fp.flat)
    assert float(st["agent_steps"]) > 0
