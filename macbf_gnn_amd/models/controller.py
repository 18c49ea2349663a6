"""Decentralised GNN controller (reference ``controller.py:10-63``).

Edge MLP 5->64->128 over the top-K neighbour graph, radius-masked max-pool, node MLP
132->64->128->64->4 and a gain-scheduled PD law. Parameter names/shapes follow the
reference (``controller_centr_net.{0,2}`` Conv1d, ``controller_dec_net.{0,2,4,6}`` Linear).

CPU: pure-torch oracle. HIP device: fused MFMA kernels (``csrc/ctrl.hip``) via an autograd
Function with hand-written backward.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import config as C
from .. import oracle


class Controller(nn.Module):
    def __init__(self, in_dim: int = 4):
        super().__init__()
        if in_dim not in (4, 6):
            raise NotImplementedError("double integrator in 2-D (in_dim=4) or 3-D (in_dim=6)")
        self.in_dim = in_dim
        self.controller_centr_net = nn.Sequential(
            nn.Conv1d(in_dim + 1, 64, (1,)), nn.ReLU(),
            nn.Conv1d(64, 128, (1,)), nn.ReLU(),
        )
        self.controller_dec_net = nn.Sequential(
            nn.Linear(128 + in_dim, 64), nn.ReLU(),
            nn.Linear(64, 128), nn.ReLU(),
            nn.Linear(128, 64), nn.ReLU(),
            nn.Linear(64, in_dim),
        )

    def params_dict(self):
        return dict(self.named_parameters())

    def forward(self, states: torch.Tensor, goals: torch.Tensor, idx: torch.Tensor | None = None,
                top_k: int = C.TOP_K, obstacles: torch.Tensor | None = None):
        """states (N,2D), goals (N,D) -> a (N,D); batched (...,N,2D),(...,N,D) -> (...,N,D).
        ``obstacles`` (M,D) / (B,M,D): static points that join the neighbour graph."""
        single = states.dim() == 2
        s = states.unsqueeze(0) if single else states
        g = goals.unsqueeze(0) if single else goals
        if s.device.type == "cpu":
            nodes = oracle.with_obstacles(s, obstacles)
            if idx is None:
                idx = oracle.knn_idx(s.detach(), top_k, nodes.detach())
            a = oracle.controller_forward(self.params_dict(), s, g, idx, nodes=nodes)
        else:
            from ..ops import ctrl as ctrl_ops
            a = ctrl_ops.controller_apply(self, s, g, idx, top_k, obstacles=obstacles)
        return a[0] if single else a
