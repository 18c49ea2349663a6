"""3-D double integrator and static obstacles (BASELINE config #5 semantics) on the CPU oracle."""
import numpy as np
import pytest
import torch

from macbf_gnn_amd import config as C
from macbf_gnn_amd import env as E
from macbf_gnn_amd import oracle as O
from macbf_gnn_amd.engine import Trainer
from macbf_gnn_amd.models import CBF, Controller
from macbf_gnn_amd.parallel import DP

CPU = torch.device("cpu")


def test_2d_paths_unchanged_by_generalisation():
    """D = 2 without obstacles: the generalised oracle is the reference formula set."""
    s, g = E.generate_batch(1, 20, seed=4)
    s[..., 2:] = torch.randn(1, 20, 2) * 0.3
    idx = O.knn_idx(s, 12)
    rel, eye = O.edge_rel(s, idx)
    d = torch.sqrt(rel[..., 0] ** 2 + rel[..., 1] ** 2 + 2e-4)
    x, mask = O.cbf_features(s, idx)
    torch.testing.assert_close(x[..., 5], d - C.DIST_MIN_THRES)
    ar = O.action_ref(s, g)
    torch.testing.assert_close(ar[..., 0], -((s[..., 0] - g[..., 0]) + C.SQRT3 * s[..., 2]))


def test_3d_scenarios_invariants():
    s, g, obs = E.generate_scenarios(2, 40, dim=3, num_obstacles=3, seed=1)
    assert s.shape == (2, 40, 6) and g.shape == (2, 40, 3) and obs.shape == (2, 36, 3)
    for b in range(2):
        p = s[b, :, :3]
        d = torch.cdist(p, p) + torch.eye(40) * 9
        assert d.min() > C.DIST_MIN_THRES
        assert torch.cdist(p, obs[b]).min() > C.DIST_MIN_THRES
        assert torch.cdist(g[b], obs[b]).min() > C.DIST_MIN_THRES
        assert torch.all((g[b] - p).abs() <= C.GOAL_SPREAD)


def test_obstacles_join_the_graph_but_not_the_agents():
    s, g, obs = E.generate_scenarios(1, 12, dim=2, num_obstacles=2, seed=3)
    nodes = O.with_obstacles(s, obs)
    assert nodes.shape == (1, 12 + 24, 4) and torch.all(nodes[0, 12:, 2:] == 0)
    idx = O.knn_idx(s, 12, nodes)
    assert idx.shape == (1, 12, 12) and torch.all(idx[0, :, 0] == torch.arange(12))
    assert (idx >= 12).any()          # some neighbour slots are obstacle points
    ctrl = Controller(4)
    a = ctrl(s, g, obstacles=obs)
    assert a.shape == (1, 12, 2)


@pytest.mark.parametrize("dim,nobs", [(3, 0), (2, 2), (3, 2)])
def test_train_step_nd_obstacles(dim, nobs):
    cfg = C.TrainConfig(num_agents=10, num_envs=2, inner_loops=4, device="cpu", seed=0, dim=dim,
                        num_obstacles=nobs)
    tr = Trainer(cfg, device=CPU, dp=DP(device=CPU))
    before = tr.fp.flat.clone()
    st = tr.train_step()
    assert torch.isfinite(torch.as_tensor(st["loss_total"]))
    assert torch.isfinite(tr.fp.flat).all() and not torch.equal(before, tr.fp.flat)
    assert sum(p.numel() for p in tr.controller.parameters()) == (
        64 * (2 * dim + 1) + 64 + 128 * 64 + 128 + 64 * (128 + 2 * dim) + 64 + 128 * 64 + 128 + 64 * 128 + 64
        + 2 * dim * 64 + 2 * dim)


def test_3d_ttc_closed_form():
    rng = np.random.default_rng(0)
    s = torch.tensor(rng.uniform(0, 1, size=(30, 6)), dtype=torch.float64)
    s[:, 3:] -= 0.5
    m = O.ttc_mask_all_pairs(s).numpy()
    for i in range(30):
        for j in range(30):
            if i == j:
                continue
            p = (s[i, :3] - s[j, :3]).numpy()
            v = (s[i, 3:] - s[j, 3:]).numpy()
            ts = np.linspace(0, C.TIME_TO_COLLISION_CHECK, 2001)
            dmin = np.min(np.linalg.norm(p[None] + v[None] * ts[:, None], axis=1))
            if abs(dmin - C.DIST_MIN_CHECK) > 1e-4:
                assert m[i, j] == (dmin < C.DIST_MIN_CHECK)
