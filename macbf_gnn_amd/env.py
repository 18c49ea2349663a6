"""Environment: obstacles, scenario sampling and double-integrator dynamics.

Host-side numpy versions reproduce the reference semantics exactly
(``/root/reference/core.py:7-86``); they are the golden path for tests and for the
single-env ``core.py`` API. The batched GPU sampler lives in
``macbf_gnn_amd.ops.scenario`` (HIP kernel ``csrc/scenario.hip``) and is checked
against the invariants of these functions.
"""
from __future__ import annotations

import numpy as np
import torch

from . import config as C


def generate_obstacle_circle(center, radius, num=12):
    """``num`` points evenly spaced on a circle (core.py:7-12)."""
    theta = np.linspace(0.0, 2.0 * np.pi, num=num, endpoint=False)
    pts = np.stack([np.cos(theta), np.sin(theta)], axis=1) * radius
    return np.asarray(center, dtype=np.float64) + pts


def generate_obstacle_rectangle(center, sides, num=12):
    """``num`` boundary points of an axis-aligned rectangle (core.py:15-42).

    Points are split over top/right/bottom/left in proportion to the side lengths
    with the same integer rounding as the reference.
    """
    a, b = sides
    n1 = int(num // 2 * a / (a + b))
    n2 = num // 2 - n1
    n3 = n1
    n4 = num - n1 - n2 - n3
    top = np.stack([np.linspace(-a / 2, a / 2, n1, endpoint=False), np.full(n1, b / 2)], 1)
    right = np.stack([np.full(n2, a / 2), np.linspace(b / 2, -b / 2, n2, endpoint=False)], 1)
    bottom = np.stack([np.linspace(a / 2, -a / 2, n3, endpoint=False), np.full(n3, -b / 2)], 1)
    left = np.stack([np.full(n4, -a / 2), np.linspace(-b / 2, b / 2, n4, endpoint=False)], 1)
    rect = np.concatenate([top, right, bottom, left], axis=0)
    return rect + np.asarray(center, dtype=np.float64)


def side_length(num_agents: int, dim: int = 2) -> float:
    """Side of the square (D=2, core.py:46) / cube (D=3) holding AGENT_DENSITY agents per unit."""
    return float(max(1.0, num_agents / C.AGENT_DENSITY) ** (1.0 / dim))


def generate_obstacle_sphere(center, radius, num=12):
    """``num`` points spread over a sphere (Fibonacci lattice): the 3-D point-set obstacle."""
    k = np.arange(num) + 0.5
    phi = np.arccos(1.0 - 2.0 * k / num)
    th = np.pi * (1.0 + 5 ** 0.5) * k
    pts = np.stack([np.cos(th) * np.sin(phi), np.sin(th) * np.sin(phi), np.cos(phi)], 1) * radius
    return np.asarray(center, dtype=np.float64) + pts


def generate_obstacles(num_obstacles, L, dim=2, rng: np.random.Generator | None = None, points=12):
    """``num_obstacles`` static point-set obstacles inside the arena -> (num_obstacles*points, D).
    D = 2: alternating circles / rectangles (the reference generators, core.py:7-42);
    D = 3: spheres."""
    rng = rng or np.random.default_rng()
    out = []
    for q in range(num_obstacles):
        c = rng.uniform(0.0, L, size=(dim,))
        if dim == 3:
            out.append(generate_obstacle_sphere(c, rng.uniform(0.1, 0.3), points))
        elif q % 2 == 0:
            out.append(generate_obstacle_circle(c, rng.uniform(0.1, 0.3), points))
        else:
            out.append(generate_obstacle_rectangle(c, rng.uniform(0.2, 0.6, size=(2,)), points))
    if not out:
        return np.zeros((0, dim), dtype=np.float32)
    return np.concatenate(out, 0).astype(np.float32)


def _rsa(n, dim, thres, sample, rng, fixed=None):
    """Sequential rejection sampling of n points, each > thres from every earlier point and
    from the fixed points (obstacles)."""
    pts = np.zeros((n, dim), dtype=np.float32)
    fixed = np.zeros((0, dim), dtype=np.float32) if fixed is None else fixed
    i = 0
    tries = 0
    while i < n:
        cand = sample(i)
        tries += 1
        prev = np.concatenate([pts[:i], fixed], 0)
        if prev.shape[0] and np.min(np.linalg.norm(prev - cand, axis=1)) <= thres:
            if tries > 1000 * n:
                raise RuntimeError("scenario sampler: arena too crowded")
            continue
        pts[i] = cand
        i += 1
    return pts


def generate_data_nd(num_agents, dim=2, dist_min_thres=C.DIST_MIN_THRES, rng=None, obstacles=None):
    """D-dimensional scenario (starts at rest, goals within GOAL_SPREAD per coordinate), with
    starts and goals kept > dist_min_thres from each other and from the obstacle points."""
    rng = rng or np.random.default_rng()
    L = side_length(num_agents, dim)
    st = _rsa(num_agents, dim, dist_min_thres, lambda i: rng.uniform(size=(dim,)) * L, rng, obstacles)
    gl = _rsa(num_agents, dim, dist_min_thres,
              lambda i: rng.uniform(-C.GOAL_SPREAD, C.GOAL_SPREAD, size=(dim,)) + st[i], rng, obstacles)
    states = np.concatenate([st, np.zeros_like(st)], 1).astype(np.float32)
    return states, gl.astype(np.float32)


def generate_scenarios(num_envs, num_agents, dim=2, num_obstacles=0, seed=0, dist_min_thres=C.DIST_MIN_THRES):
    """Host sampler for batched D-dimensional scenarios with obstacles ->
    (s (B,N,2D), g (B,N,D), obs (B,M,D) or None). D = 2 without obstacles is ``generate_batch``."""
    if dim == 2 and num_obstacles == 0:
        s, g = generate_batch(num_envs, num_agents, dist_min_thres, seed)
        return s, g, None
    rng = np.random.default_rng(seed)
    S, G, O = [], [], []
    for _ in range(num_envs):
        obs = generate_obstacles(num_obstacles, side_length(num_agents, dim), dim, rng)
        s_, g_ = generate_data_nd(num_agents, dim, dist_min_thres, rng, obs if num_obstacles else None)
        S.append(s_); G.append(g_); O.append(obs)
    obs_t = torch.from_numpy(np.stack(O)) if num_obstacles else None
    return torch.from_numpy(np.stack(S)), torch.from_numpy(np.stack(G)), obs_t


def generate_data(num_agents, dist_min_thres, rng: np.random.Generator | None = None):
    """Sequential rejection sampling of starts and goals (core.py:45-71).

    Keeps the reference quirk that not-yet-filled rows are zeros and take part in the
    min-distance test, so nothing is placed within ``dist_min_thres`` of the origin.
    Returns ``states (N,4) float32`` (zero velocity) and ``goals (N,2) float32``.
    """
    uniform = (rng.uniform if rng is not None else np.random.uniform)
    L = side_length(num_agents)
    states = np.zeros((num_agents, 2), dtype=np.float32)
    goals = np.zeros((num_agents, 2), dtype=np.float32)
    i = 0
    while i < num_agents:
        cand = uniform(size=(2,)) * L
        if np.min(np.linalg.norm(states - cand, axis=1)) <= dist_min_thres:
            continue
        states[i] = cand
        i += 1
    i = 0
    while i < num_agents:
        cand = uniform(-C.GOAL_SPREAD, C.GOAL_SPREAD, size=(2,)) + states[i]
        if np.min(np.linalg.norm(goals - cand, axis=1)) <= dist_min_thres:
            continue
        goals[i] = cand
        i += 1
    states = np.concatenate([states, np.zeros((num_agents, 2), dtype=np.float32)], axis=1)
    return states, goals


def generate_batch(num_envs, num_agents, dist_min_thres=C.DIST_MIN_THRES, seed=0):
    """Host reference sampler for ``num_envs`` independent scenarios -> (B,N,4), (B,N,2)."""
    rng = np.random.default_rng(seed)
    s, g = zip(*[generate_data(num_agents, dist_min_thres, rng) for _ in range(num_envs)])
    return torch.from_numpy(np.stack(s)), torch.from_numpy(np.stack(g))


def dynamics(states, actions):
    """2-D double integrator ds/dt = [vx, vy, ax, ay] (core.py:74-86); any leading dims."""
    return torch.cat([states[..., 2:], actions], dim=-1)


def euler_step(states, actions, dt=C.TIME_STEP):
    return states + dynamics(states, actions) * dt
