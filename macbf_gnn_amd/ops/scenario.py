"""Batched on-device scenario sampler (HIP kernel ``csrc/scenario.hip``).

Counter-based RNG: scenarios depend only on (seed, iteration, rank, env), so resuming from a
checkpoint at any DP width reproduces the data stream without saving RNG state.
"""
from __future__ import annotations

import torch

from .. import config as C
from .. import env as E
from . import host, native


def _mix(*xs) -> int:
    h = 0x9E3779B97F4A7C15
    for x in xs:
        h ^= (int(x) + 0x9E3779B97F4A7C15 + ((h << 6) & 0xFFFFFFFFFFFFFFFF) + (h >> 2)) & 0xFFFFFFFFFFFFFFFF
        h = (h * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    return h


def iteration_key(seed, iteration, rank, salt=0) -> int:
    """Signed 64-bit counter-based RNG key of (seed, iteration, rank[, salt]) (device int64)."""
    k = _mix(seed, iteration, rank, salt) if salt else _mix(seed, iteration, rank)
    return k - (1 << 64) if k >= (1 << 63) else k


def obstacles(B, N, *, dim, num_obstacles, points, seed, device):
    """(B, num_obstacles*points, D) static point-set obstacles with the shapes of
    ``env.generate_obstacles`` (2-D: alternating circles / rectangles, 3-D: spheres), from the
    counter-based host sampler (``ops.host``; a few hundred floats) -> identical on CPU and GPU
    for one seed; copied to the device asynchronously from pinned memory."""
    pin = torch.device(device).type == "cuda"
    out = torch.empty(B, num_obstacles * points, dim, dtype=torch.float32, pin_memory=pin)
    host.sample_obstacles(B, N, dim=dim, num_obstacles=num_obstacles, points=points, seed=seed, out=out)
    return out.to(device, non_blocking=True) if pin else out


def generate(B, N, *, seed=0, iteration=0, rank=0, device=None, out=None, dim=2, num_obstacles=0,
             obstacle_points=12):
    """-> (s0 (B,N,2D), g (B,N,D), obstacles (B,M,D) or None). HIP device: the on-device
    parallel RSA kernel; CPU: the same process in the host runtime (bit-identical output).
    Obstacle points are fixed conflict points for starts and goals."""
    device = torch.device(device or "cuda")
    key = _mix(seed, iteration, rank)
    obs = None
    if num_obstacles:
        obs = obstacles(B, N, dim=dim, num_obstacles=num_obstacles, points=obstacle_points, seed=key ^ 0x5EED,
                        device=device)
    if device.type != "cuda":
        s0, g, _ = host.sample_scenarios(B, N, dim=dim, seed=key, obs=obs)
        return s0, g, obs
    W = native.rec_width(dim)
    if out is None or dim != 2:
        S = torch.empty(B, N, W, dtype=torch.float32, device=device)
        G = torch.empty(B, N, dim, dtype=torch.float32, device=device)
    else:
        S, G = out
    native.scenario(S, G, seed=key, L=E.side_length(N, dim), r=C.DIST_MIN_THRES, spread=C.GOAL_SPREAD, obs=obs)
    return native.from_records(S), G, obs
