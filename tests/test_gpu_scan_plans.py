"""Every production instantiation of the kNN / TTC / safety scan, pinned to the fp32 oracle with
a temporal bound.

The launcher picks the block size, the lanes per agent and the cell grid from the call's shape
(csrc/scan.hip launch_kd / plan_kdb). Each case below first asserts, through
``native.scan_plan``, that it hits the instantiation it names, then runs >= 3 steps on moving
states with the previous step's kNN as the bound (the cell-grid search) and compares the lists,
danger bits, counts and safety counts with the oracle (reference semantics: /root/reference
core.py:187-209 kNN + TTC mask, core.py:234-250 safety check). ``lattice`` rounds the positions
to a coarse grid: many exactly equal distances, so the (distance, index) tie order is checked.

Negative check (one-off, recorded in profiles/r6_runs/r6c/neg.log: 12 of 12 fail): the same tests run against a build
whose cell search box is shrunk to 0.7x (``scripts/build_variant.sh shrink scan "-DMB_DIAG=8"``).
"""
import pytest
import torch

from macbf_gnn_amd import config as C
from macbf_gnn_amd import oracle as O
from macbf_gnn_amd.ops import native

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")

# (name, B, agents, dim, obstacle points, lanes, expected plan)
PLANS = [
    # BASELINE config #3 headline: 1024-thread blocks, 4 lanes per agent, 24^2 cell grid
    ("headline_2d", 64, 1024, 2, 0, 0, dict(bs=1024, lpa=4, glb=0, use_cells=1, cell_g=24, wave_atomic=0)),
    # config #5: 3-D, 8 obstacles x 12 points, 512-thread blocks, per-wave count atomics, 10^3 grid
    ("cfg5_3d_obstacles", 64, 1024, 3, 96, 0, dict(bs=512, lpa=4, glb=0, use_cells=1, cell_g=10, wave_atomic=1)),
    # the DP=8 slice of config #3 (8 envs per rank): 256-thread blocks, 8 lanes per agent, 16^2 grid
    ("slice8_2d", 8, 1024, 2, 0, 0, dict(bs=256, lpa=8, glb=0, use_cells=1, cell_g=16, wave_atomic=0)),
    # small 3-D scenes: 256-thread blocks with 4 cells per thread in the prefix sum,
    # at the auto layout (8 lanes) and forced 4 lanes
    ("small_3d_auto", 2, 300, 3, 0, 0, dict(bs=256, lpa=8, glb=0, use_cells=1, cell_g=10, wave_atomic=1)),
    ("small_3d_lanes4", 2, 300, 3, 24, 4, dict(bs=256, lpa=4, glb=0, use_cells=1, cell_g=10, wave_atomic=1)),
]


def _scene(B, N, dim, M, seed, lattice):
    """Agents uniform at the trainer's density (AGENT_DENSITY per unit area / volume, the cell
    sort's domain), velocities up to 1 per axis (large steps: the lists change between steps),
    M static obstacle points per env."""
    g = torch.Generator().manual_seed(seed)
    L = max(1.0, N / C.AGENT_DENSITY) ** (1.0 / dim)
    p = torch.rand(B, N, dim, generator=g) * L
    v = (torch.rand(B, N, dim, generator=g) - 0.5) * 2.0
    if lattice:
        p = torch.round(p * 2) / 2
    obs = torch.rand(B, M, dim, generator=g) * L if M else None
    if lattice and obs is not None:
        obs = torch.round(obs * 2) / 2
    return torch.cat([p, v], -1).to(DEV), (obs.to(DEV) if obs is not None else None)


def _records(s, obs):
    nodes = O.with_obstacles(s, obs)
    return native.to_records(nodes), nodes


@pytest.mark.parametrize("lattice", [False, True])
@pytest.mark.parametrize("name,B,N,dim,M,lanes,want", PLANS, ids=[p[0] for p in PLANS])
def test_scan_production_plan_matches_oracle(name, B, N, dim, M, lanes, want, lattice):
    K = C.TOP_K
    Nn = N + M
    plan = native.scan_plan(B, N, K, Nn=Nn, dim=dim, prev=True, lanes=lanes)
    for k, v in want.items():
        assert plan[k] == v, (name, k, plan)
    first = native.scan_plan(B, N, K, Nn=Nn, dim=dim, prev=False, lanes=lanes)
    assert first["bs"] == want["bs"] and first["lpa"] == want["lpa"] and first["cells"] == 0, first
    s, obs = _scene(B, N, dim, M, seed=sum(map(ord, name)) + int(lattice), lattice=lattice)
    prev = None
    for step in range(4):
        S, nodes = _records(s, obs)
        idx = torch.empty(B, N, K, dtype=torch.int32, device=DEV)
        dang = torch.empty(B, N, K, dtype=torch.uint8, device=DEV)
        cnt = torch.zeros(B, 2, device=DEV)
        safe = torch.zeros(B, device=DEV)
        native.scan(S, idx, dang, cnt, safe, K=K, n_agents=N, prev_idx=prev, sort=step % 2 == 0, lanes=lanes)
        torch.cuda.synchronize()
        ref = O.knn_idx(s, K, nodes)
        bad = (idx.long() != ref).any(-1)
        assert not bad.any(), (name, step, int(bad.sum()))
        dref = O.ttc_mask_knn(s, ref, nodes)
        assert torch.equal(dang.bool(), dref), (name, step)
        assert torch.equal(cnt[:, 0], dref.sum((1, 2)).float()), (name, step)
        assert torch.equal(cnt[:, 1], (~dref).sum((1, 2)).float()), (name, step)
        assert torch.equal(safe, O.safe_agent_count(s, nodes).float()), (name, step)
        prev = idx
        dim_ = s.shape[-1] // 2
        s = (s + torch.cat([s[..., dim_:], torch.zeros_like(s[..., dim_:])], -1) * 0.1).contiguous()
        if lattice:     # keep the tie structure while moving
            s[..., :dim_] = torch.round(s[..., :dim_] * 2) / 2

