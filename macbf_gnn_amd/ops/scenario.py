"""Batched on-device scenario sampler (HIP kernel ``csrc/scenario.hip``).

Counter-based RNG: scenarios depend only on (seed, iteration, rank, env), so resuming from a
checkpoint at any DP width reproduces the data stream without saving RNG state.
"""
from __future__ import annotations

import torch

from .. import config as C
from .. import env as E
from . import native


def _mix(*xs) -> int:
    h = 0x9E3779B97F4A7C15
    for x in xs:
        h ^= (int(x) + 0x9E3779B97F4A7C15 + ((h << 6) & 0xFFFFFFFFFFFFFFFF) + (h >> 2)) & 0xFFFFFFFFFFFFFFFF
        h = (h * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    return h


def generate(B, N, *, seed=0, iteration=0, rank=0, device=None, out=None, dim=2, num_obstacles=0,
             obstacle_points=12):
    """-> (s0 (B,N,2D), g (B,N,D), obstacles (B,M,D) or None)."""
    device = device or torch.device("cuda")
    if dim != 2 or num_obstacles:
        raise NotImplementedError("on-device sampler: 2-D without obstacles (3-D / obstacles: see generate_nd)")
    if out is None:
        S = torch.empty(B, N, 4, dtype=torch.float32, device=device)
        G = torch.empty(B, N, 2, dtype=torch.float32, device=device)
    else:
        S, G = out
    native.scenario(S, G, seed=_mix(seed, iteration, rank), L=E.side_length(N), r=C.DIST_MIN_THRES,
                    spread=C.GOAL_SPREAD)
    return S, G, None
