"""Host (CPU) native runtime ``macbf_gnn_amd._host`` (plain C++, ``csrc/host``).

* ``sample_scenarios``: the parallel random-sequential-adsorption sampler of the device kernel
  (``csrc/scenario.hip``) with identical proposals and acceptance rule, O(N) per round via a
  uniform grid and threaded over environments -- CPU and GPU trainers see bit-identical data
  for one seed (tested on the GPU).
* ``sample_obstacles``: counter-based static point-set obstacles (used by both paths).

The module is built in-tree by ``csrc/build.py``; when it is missing (a fresh CPU checkout)
only the host target is compiled with g++ on first use. Every wrapper validates dtype, device,
contiguity and shape before handing raw addresses to C++.
"""
from __future__ import annotations

import math
import os
import subprocess
import sys
from typing import Optional

import numpy as np
import torch

from .. import config as C
from .. import env as E

_LIB = None


def _build_host():
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.join(root, "csrc"))
    try:
        import build as B  # csrc/build.py
    finally:
        sys.path.pop(0)
    B.write_ninja()
    r = subprocess.run(["ninja", "-C", B.BUILD, B.host_ext_path()], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("host runtime build failed:\n" + r.stdout + r.stderr)


def lib():
    global _LIB
    if _LIB is None:
        try:
            from .. import _host
        except ImportError:
            _build_host()
            from .. import _host
        _LIB = _host
    return _LIB


def _chk(t, shape, dtype=torch.float32, name="tensor"):
    if t.device.type != "cpu" or t.dtype != dtype or not t.is_contiguous() or tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: expected contiguous CPU {dtype} {tuple(shape)}, got {t.dtype} "
                         f"{tuple(t.shape)} on {t.device}")


def _templates(points: int):
    circ = np.stack([np.cos(np.arange(points) * (2 * np.pi / points)),
                     np.sin(np.arange(points) * (2 * np.pi / points))], 1)
    rect = E.generate_obstacle_rectangle((0.0, 0.0), (1.0, 1.0), points)
    sph = E.generate_obstacle_sphere((0.0, 0.0, 0.0), 1.0, points)
    f = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32))
    return f(circ), f(rect), f(sph)


def sample_obstacles(B: int, N: int, *, dim: int, num_obstacles: int, points: int = 12, seed: int = 0,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """(B, num_obstacles * points, dim) float32 CPU tensor (pinned when ``out`` is)."""
    M = num_obstacles * points
    if out is None:
        out = torch.empty(B, M, dim, dtype=torch.float32)
    _chk(out, (B, M, dim), name="obstacles")
    circ, rect, sph = _templates(points)
    rc = lib().sample_obstacles(out.data_ptr(), B, num_obstacles, points, dim, float(E.side_length(N, dim)),
                                seed & 0xFFFFFFFFFFFFFFFF, circ.data_ptr(), rect.data_ptr(), sph.data_ptr())
    if rc != 0:
        raise ValueError("sample_obstacles: invalid arguments")
    return out


def sample_scenarios(B: int, N: int, *, dim: int = 2, seed: int = 0, obs: Optional[torch.Tensor] = None,
                     r: float = C.DIST_MIN_THRES, spread: float = C.GOAL_SPREAD, max_rounds: int = 256,
                     threads: int = 0):
    """-> (s0 (B, N, 2*dim), g (B, N, dim), status (B,) int32): the device sampler's process on
    the host. ``status`` = goal-phase rounds used (> 0) or -1 when ``max_rounds`` was hit."""
    S = torch.empty(B, N, 2 * dim, dtype=torch.float32)
    G = torch.empty(B, N, dim, dtype=torch.float32)
    st = torch.zeros(B, dtype=torch.int32)
    M = 0
    if obs is not None:
        M = obs.shape[1]
        _chk(obs, (B, M, dim), name="obs")
    rc = lib().sample_scenarios(S.data_ptr(), G.data_ptr(), obs.data_ptr() if obs is not None else 0, st.data_ptr(),
                                B, N, dim, M, float(E.side_length(N, dim)), float(r), float(spread),
                                seed & 0xFFFFFFFFFFFFFFFF, int(max_rounds), int(threads))
    if rc != 0:
        raise ValueError("sample_scenarios: invalid arguments")
    return S, G, st


def min_pair_distance(p: torch.Tensor, cutoff: float = 1.0) -> float:
    """Minimum pairwise distance of the (n, dim) points (capped at ``cutoff``), O(n)."""
    p = p.detach().float().contiguous().cpu()
    n, dim = p.shape
    L = float(p.max().item()) + 1.0 if n else 1.0
    return float(lib().min_pair_distance(p.data_ptr(), n, dim, dim, L, float(cutoff)))
