"""Decentralised neural control barrier function (reference ``cbf.py:8-45``).

Parameter names and shapes are the reference's (``cbf_net.{0,2,4,6}.{weight,bias}`` with
Conv1d(k=1) weights of shape (out, in, 1)), so reference ``state_dict``s load unchanged.

``forward`` evaluates h on the kNN graph:
* on CPU: the pure-torch oracle (``macbf_gnn_amd.oracle.cbf_forward``);
* on a HIP device: the fused MFMA edge-MLP kernels (``csrc/cbf.hip``) through an autograd
  Function with a hand-written backward. There is no silent fallback: a missing native
  extension on a GPU raises.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import config as C
from .. import oracle


class CBF(nn.Module):
    def __init__(self, in_dim: int = 4):
        super().__init__()
        if in_dim not in (4, 6):
            raise NotImplementedError("double integrator in 2-D (in_dim=4) or 3-D (in_dim=6)")
        self.in_dim = in_dim
        self.cbf_net = nn.Sequential(
            nn.Conv1d(in_dim + 2, 64, (1,)), nn.ReLU(),
            nn.Conv1d(64, 128, (1,)), nn.ReLU(),
            nn.Conv1d(128, 64, (1,)), nn.ReLU(),
            nn.Conv1d(64, 1, (1,)),
        )

    def params_dict(self):
        return dict(self.named_parameters())

    def forward(self, states: torch.Tensor, idx: torch.Tensor | None = None, top_k: int = C.TOP_K,
                obstacles: torch.Tensor | None = None):
        """states (N,2D) -> h (N,1,K) [reference layout]; states (...,N,2D) -> h (...,N,K).
        ``obstacles`` (M,D) / (B,M,D): static points that join the neighbour graph."""
        single = states.dim() == 2
        s = states.unsqueeze(0) if single else states
        if s.device.type == "cpu":
            nodes = oracle.with_obstacles(s, obstacles)
            if idx is None:
                idx = oracle.knn_idx(s.detach(), top_k, nodes.detach())
            h = oracle.cbf_forward(self.params_dict(), s, idx, nodes=nodes)
        else:
            from ..ops import cbf as cbf_ops
            h = cbf_ops.cbf_apply(self, s, idx, top_k, obstacles=obstacles)
        if single:
            return h[0].unsqueeze(1)          # (N, 1, K)
        return h
