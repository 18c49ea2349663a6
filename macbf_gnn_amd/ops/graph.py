"""Graph construction on the HIP device (K1): kNN neighbour slots of a batch of scenes."""
from __future__ import annotations

from typing import Optional

import torch

from .. import oracle
from . import native


def node_records(s: torch.Tensor, obstacles: Optional[torch.Tensor] = None) -> torch.Tensor:
    """(B, N, 2D) agent states (+ (B, M, D) static obstacle points) -> (B, N+M, W) kernel records."""
    return native.to_records(oracle.with_obstacles(s.detach().float(), obstacles))


def knn(s: torch.Tensor, k: int, obstacles: Optional[torch.Tensor] = None) -> torch.Tensor:
    """s (B, N, 2D) fp32 on the device -> idx (B, N, k) int32 into the graph nodes (agents, then
    obstacle points), nearest first, self at slot 0 (ties -> lower index; = ``oracle.knn_idx``)."""
    if s.dim() != 3:
        raise ValueError("s must be (B, N, 2D)")
    S = node_records(s, obstacles)
    B, N = s.shape[:2]
    k = min(k, S.shape[1])
    idx = torch.empty(B, N, k, dtype=torch.int32, device=s.device)
    native.scan(S, idx, None, None, None, K=k, do_knn=True, do_safety=False, n_agents=N)
    return idx


def safe_agent_count(s: torch.Tensor, obstacles: Optional[torch.Tensor] = None) -> torch.Tensor:
    """All-pairs TTC check (r=DIST_MIN_CHECK, ttc=TIME_TO_COLLISION_CHECK) of every agent against
    every node: per-env number of agents with no dangerous pair (``core.py:212-231`` +
    ``train.py:74-75``)."""
    S = node_records(s, obstacles)
    B, N = s.shape[:2]
    safe = torch.zeros(B, dtype=torch.float32, device=s.device)
    native.scan(S, None, None, None, safe, K=1, do_knn=False, do_safety=True, n_agents=N)
    return safe
