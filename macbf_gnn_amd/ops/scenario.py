"""Batched on-device scenario sampler (HIP kernel ``csrc/scenario.hip``).

Counter-based RNG: scenarios depend only on (seed, iteration, rank, env), so resuming from a
checkpoint at any DP width reproduces the data stream without saving RNG state.
"""
from __future__ import annotations

import math

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


def obstacles(B, N, *, dim, num_obstacles, points, seed, device):
    """(B, num_obstacles*points, D) static point-set obstacles with the shapes of
    ``env.generate_obstacles`` (2-D: alternating circles / rectangles, 3-D: spheres), sampled with
    device-side torch ops from a counter-based seed (no host work, stream-ordered)."""
    gen = torch.Generator(device=device)
    gen.manual_seed(seed & 0x7FFFFFFFFFFFFFFF)
    L = E.side_length(N, dim)
    f32 = torch.float32
    ctr = torch.rand(B, num_obstacles, 1, dim, generator=gen, device=device, dtype=f32) * L
    if dim == 3:
        k = torch.arange(points, device=device, dtype=f32) + 0.5
        phi = torch.arccos(1.0 - 2.0 * k / points)
        th = math.pi * (1.0 + 5 ** 0.5) * k
        unit = torch.stack([torch.cos(th) * torch.sin(phi), torch.sin(th) * torch.sin(phi), torch.cos(phi)], -1)
        rad = 0.1 + 0.2 * torch.rand(B, num_obstacles, 1, 1, generator=gen, device=device, dtype=f32)
        pts = ctr + unit * rad
    else:
        th = torch.arange(points, device=device, dtype=f32) * (2.0 * math.pi / points)
        circ = torch.stack([torch.cos(th), torch.sin(th)], -1)                       # (P, 2)
        rad = 0.1 + 0.2 * torch.rand(B, num_obstacles, 1, 1, generator=gen, device=device, dtype=f32)
        sides = 0.2 + 0.4 * torch.rand(B, num_obstacles, 1, 2, generator=gen, device=device, dtype=f32)
        # rectangle boundary: the reference's proportional split, on the unit square, then scaled
        rect = torch.as_tensor(E.generate_obstacle_rectangle((0.0, 0.0), (1.0, 1.0), points), device=device,
                               dtype=f32)
        is_circ = (torch.arange(num_obstacles, device=device) % 2 == 0).view(1, -1, 1, 1)
        pts = ctr + torch.where(is_circ, circ * rad, rect * sides)
    return pts.reshape(B, num_obstacles * points, dim).contiguous()


def generate(B, N, *, seed=0, iteration=0, rank=0, device=None, out=None, dim=2, num_obstacles=0,
             obstacle_points=12):
    """-> (s0 (B,N,2D), g (B,N,D), obstacles (B,M,D) or None): on-device parallel RSA; obstacle
    points are fixed conflict points for starts and goals."""
    device = device or torch.device("cuda")
    key = _mix(seed, iteration, rank)
    obs = None
    if num_obstacles:
        obs = obstacles(B, N, dim=dim, num_obstacles=num_obstacles, points=obstacle_points, seed=key ^ 0x5EED,
                        device=device)
    W = native.rec_width(dim)
    if out is None or dim != 2:
        S = torch.empty(B, N, W, dtype=torch.float32, device=device)
        G = torch.empty(B, N, dim, dtype=torch.float32, device=device)
    else:
        S, G = out
    native.scenario(S, G, seed=key, L=E.side_length(N, dim), r=C.DIST_MIN_THRES, spread=C.GOAL_SPREAD, obs=obs)
    return native.from_records(S), G, obs
