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


def side_length(num_agents: int) -> float:
    return float(np.sqrt(max(1.0, num_agents / C.AGENT_DENSITY)))


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
