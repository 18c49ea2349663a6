"""Deduplicated h / h' evaluations: pure-torch reference of ``csrc/dedup.hip``.

The derivative loss (reference ``core.py:132-171``) needs h'(s_{t+1}) of every kNN slot
(t, b, i, k) on the time-t neighbour j = idx_t[i, k] (reuse_nbr_idx). The barrier
network is a function of the pair's relative state only (``cbf.py:21-45``), so h' of that slot
equals h of the slot (t+1, b, i, k') of the same pair, whenever j is still one of i's
neighbours at t+1. Only the unmatched pairs (and the whole last step) need an extra
evaluation. ``match_reference`` builds the same index maps as the HIP kernel:

* ``map1[t, b, i, k]``: evaluation index of the h' partner of main slot e (< E: a main slot of
  step t+1; >= E: an extra evaluation, ordered by (t, b, i, k));
* ``src[u]``: the main slot whose h' is evaluation u (or -1);
* ``nev``: number of evaluations U = E + extras.
"""
from __future__ import annotations

import torch


def match_reference(idx: torch.Tensor, T: int, recomputed: bool = False):
    """idx (>= T + recomputed, B, N, K) -> (map1 (T,B,N,K), src (2E,), nev) as int64 tensors."""
    _, B, N, K = idx.shape
    E = T * B * N * K
    BNK = B * N * K
    idx = idx.long().cpu()
    map1 = torch.full((T, B, N, K), -1, dtype=torch.long)
    src = torch.full((2 * E,), -1, dtype=torch.long)
    x = E
    for t in range(T):
        cur = idx[t]
        for b in range(B):
            for i in range(N):
                for k in range(K):
                    e = ((t * B + b) * N + i) * K + k
                    m = -1
                    if t + 1 < T:
                        if recomputed:
                            m = k
                        else:
                            hits = (idx[t + 1, b, i] == cur[b, i, k]).nonzero()
                            m = int(hits[-1]) if len(hits) else -1
                    if m >= 0:
                        u = e + BNK - k + m
                        map1[t, b, i, k] = u
                        src[u] = e
                    else:
                        map1[t, b, i, k] = x
                        src[x] = e
                        x += 1
    return map1, src, x


def extras_fraction(idx: torch.Tensor, T: int) -> float:
    """Fraction of main slots whose neighbour leaves the list at the next step (+ last step)."""
    a, b = idx[: T - 1].long(), idx[1:T].long()
    kept = (a.unsqueeze(-1) == b.unsqueeze(-2)).any(-1)
    E = idx[:T].numel()
    return float((~kept).sum() + idx[T - 1].numel()) / E
