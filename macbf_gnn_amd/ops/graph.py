"""Graph construction on the HIP device (K1): kNN neighbour slots of a batch of scenes."""
from __future__ import annotations

import torch

from . import native


def knn(s: torch.Tensor, k: int) -> torch.Tensor:
    """s (B, N, 4) fp32 on the device -> idx (B, N, k) int32, nearest first, self at slot 0
    (ties -> lower index; identical to ``oracle.knn_idx``)."""
    if s.dim() != 3 or s.shape[-1] != 4:
        raise ValueError("s must be (B, N, 4)")
    s = s.detach().float().contiguous()
    B, N, _ = s.shape
    k = min(k, N)
    idx = torch.empty(B, N, k, dtype=torch.int32, device=s.device)
    native.scan(s, idx, None, None, None, K=k, do_knn=True, do_safety=False)
    return idx


def safe_agent_count(s: torch.Tensor) -> torch.Tensor:
    """All-pairs TTC check (r=DIST_MIN_CHECK, ttc=TIME_TO_COLLISION_CHECK): per-env number of
    agents with no dangerous pair (reference ``core.py:212-231`` + ``train.py:74-75``)."""
    s = s.detach().float().contiguous()
    B, N, _ = s.shape
    safe = torch.zeros(B, dtype=torch.float32, device=s.device)
    native.scan(s, None, None, None, safe, K=1, do_knn=False, do_safety=True)
    return safe
