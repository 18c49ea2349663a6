"""Host (CPU) native runtime ``csrc/host``: sanitizer self-test build,
sampler invariants, determinism and the CPU trainer's data path."""
import os
import shutil
import subprocess

import numpy as np
import pytest
import torch

from macbf_gnn_amd import config as C
from macbf_gnn_amd import env as E
from macbf_gnn_amd.ops import host, scenario

HOST = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc", "host")


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
@pytest.mark.timeout(300)
def test_host_runtime_selftest_under_asan_ubsan(tmp_path):
    """The C++ sampler's own invariant checks, built with AddressSanitizer + UBSan."""
    exe = str(tmp_path / "selftest")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-ffp-contract=off", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", f"-I{HOST}",
           os.path.join(HOST, "selftest.cpp"), os.path.join(HOST, "scenario_host.cpp"), "-o", exe, "-pthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("dim,N,nobs", [(2, 1, 0), (2, 8, 0), (2, 256, 2), (3, 200, 3)])
def test_host_sampler_invariants(dim, N, nobs):
    B = 3
    obs = host.sample_obstacles(B, N, dim=dim, num_obstacles=nobs, seed=9) if nobs else None
    s, g, st = host.sample_scenarios(B, N, dim=dim, seed=17, obs=obs)
    L = E.side_length(N, dim)
    assert s.shape == (B, N, 2 * dim) and g.shape == (B, N, dim)
    assert (st > 0).all()
    assert torch.all(s[..., dim:] == 0)
    assert torch.all((s[..., :dim] >= 0) & (s[..., :dim] <= L))
    assert torch.all((g - s[..., :dim]).abs() <= C.GOAL_SPREAD + 1e-6)
    for b in range(B):
        for pts in (s[b, :, :dim], g[b]):
            if N > 1:
                d = torch.cdist(pts.double(), pts.double()) + torch.eye(N, dtype=torch.float64) * 9
                assert d.min() > C.DIST_MIN_THRES
                assert abs(host.min_pair_distance(pts) - min(float(d.min()), 1.0)) < 1e-5
            if obs is not None:
                assert torch.cdist(pts.double(), obs[b].double()).min() > C.DIST_MIN_THRES


def test_host_sampler_deterministic_and_thread_independent():
    a = host.sample_scenarios(6, 300, seed=5, threads=1)
    b = host.sample_scenarios(6, 300, seed=5, threads=4)
    c = host.sample_scenarios(6, 300, seed=6, threads=4)
    assert all(torch.equal(x, y) for x, y in zip(a, b))
    assert not torch.equal(a[0], c[0])


def test_host_obstacles_have_reference_shapes():
    """Each obstacle is centre + scale * unit template of env.generate_obstacle_* (2-D circles
    and rectangles alternate, 3-D spheres)."""
    o = host.sample_obstacles(2, 64, dim=2, num_obstacles=4, points=12, seed=1).view(2, 4, 12, 2).double()
    circ = E.generate_obstacle_circle((0.0, 0.0), 1.0, 12)
    rect = E.generate_obstacle_rectangle((0.0, 0.0), (1.0, 1.0), 12)
    for b in range(2):
        for k in range(4):
            pts = o[b, k].numpy()
            tpl = circ if k % 2 == 0 else rect
            ctr = pts.mean(0) - tpl.mean(0) * (np.ptp(pts, 0) / np.ptp(tpl, 0))
            scale = np.ptp(pts, 0) / np.ptp(tpl, 0)
            assert np.allclose(ctr + tpl * scale, pts, atol=1e-5)
            if k % 2 == 0:
                assert 0.1 - 1e-6 <= scale[0] <= 0.3 + 1e-6 and abs(scale[0] - scale[1]) < 1e-5
    o3 = host.sample_obstacles(1, 64, dim=3, num_obstacles=2, seed=2).view(2, 12, 3).double()
    for k in range(2):
        c = o3[k].mean(0)
        rad = (o3[k] - c).norm(dim=-1)
        assert rad.std() < 0.02 * rad.mean() + 1e-4


def test_cpu_trainer_uses_host_sampler():
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.parallel import DP
    cfg = C.TrainConfig(num_agents=16, num_envs=2, inner_loops=3, device="cpu", seed=4, dim=3, num_obstacles=1)
    tr = Trainer(cfg, device=torch.device("cpu"), dp=DP(device=torch.device("cpu")))
    s, g, obs = tr.sample(7)
    s2, g2, obs2 = scenario.generate(2, 16, seed=4, iteration=7, rank=0, device="cpu", dim=3, num_obstacles=1)
    assert torch.equal(s, s2) and torch.equal(g, g2) and torch.equal(obs, obs2)
    assert s.shape == (2, 16, 6) and obs.shape == (2, 12, 3)
