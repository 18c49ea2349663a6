"""Reference-compatible ``core`` module (``/root/reference/core.py``), single environment.

Every public function of the reference with its signature and return shapes, implemented
with the intended semantics of SURVEY.md section 2.4 (the reference itself does not run).
Thin wrappers over the batched engine in :mod:`macbf_gnn_amd`.
"""
from __future__ import annotations

import numpy as np
import torch

from macbf_gnn_amd import oracle as _O
from macbf_gnn_amd.config import *  # noqa: F401,F403
from macbf_gnn_amd.config import (DIST_MIN_CHECK, DIST_MIN_THRES, TIME_STEP, ALPHA_CBF, TOP_K,
                                  TIME_TO_COLLISION_CHECK, LOSS_EPS_DANG)
from macbf_gnn_amd.env import (generate_obstacle_circle, generate_obstacle_rectangle,  # noqa: F401
                               generate_data)


def dynamics(states, actions):
    """(N,4),(N,2) -> ds/dt (N,4) for the double integrator (core.py:74-86)."""
    return torch.cat([states[..., 2:], actions], dim=-1)


def remove_distant_agents(x: torch.Tensor, k: int):
    """Keep the k nearest entries of a pairwise tensor (core.py:234-250).

    ``x`` is (N, N, C) with ``x[i, j, :2]`` the relative position. Returns the gathered
    (N, K, C) tensor and the (N*K, 2) ``[row, col]`` indices, nearest first (self at slot 0
    when x[i,i,:2] = 0). Always returns the tuple, with K = min(N, k) (defect D3).
    """
    n, _, c = x.shape
    kk = min(n, k)
    d2 = x[:, :, 0] * x[:, :, 0] + x[:, :, 1] * x[:, :, 1]
    cols = torch.sort(d2, dim=1, stable=True).indices[:, :kk]
    rows = torch.arange(n, device=x.device).unsqueeze(1).expand(n, kk)
    indices = torch.stack([rows.reshape(-1), cols.reshape(-1)], dim=1)
    gathered = x[indices[:, 0], indices[:, 1]].reshape(n, kk, c)
    return gathered, indices


def _knn(states):
    if states.is_cuda:
        from macbf_gnn_amd.ops import graph
        return graph.knn(states.detach().unsqueeze(0), TOP_K)[0].long()
    return _O.knn_idx(states.detach().unsqueeze(0), TOP_K)[0]


def ttc_dangerous_mask(s):
    """Top-K time-to-collision danger mask (core.py:187-209) -> (N, K, 1) bool."""
    idx = _knn(s)
    return _O.ttc_mask_knn(s.unsqueeze(0), idx.unsqueeze(0))[0].unsqueeze(-1)


def ttc_dangerous_mask_np(s):
    """All-pairs check mask with DIST_MIN_CHECK / TIME_TO_COLLISION_CHECK (core.py:212-231)."""
    s = np.asarray(s)
    sd = np.expand_dims(s, 1) - np.expand_dims(s, 0)
    x, y, vx, vy = np.split(sd, 4, axis=2)
    eye = np.expand_dims(np.eye(s.shape[0]), 2)
    x = x + eye
    y = y + eye
    alpha = vx ** 2 + vy ** 2
    beta = 2 * (x * vx + y * vy)
    gamma = x ** 2 + y ** 2 - DIST_MIN_CHECK ** 2
    disc = beta ** 2 - 4 * alpha * gamma
    two_pos = np.logical_and(disc > 0, np.logical_and(gamma > 0, beta < 0))
    lt = np.logical_or(-beta - 2 * alpha * TIME_TO_COLLISION_CHECK < 0,
                       (beta + 2 * alpha * TIME_TO_COLLISION_CHECK) ** 2 < disc)
    return np.logical_or(gamma < 0, np.logical_and(two_pos, lt))


def _flat_h(h):
    return h.reshape(h.shape[0], -1) if h.dim() == 3 else h


def _masked_terms(v, dang, eps_d, ge_d):
    """Shared body of loss_barrier / loss_derivatives without dynamic shapes (no host sync)."""
    dm = dang.to(v.dtype)
    sm = 1.0 - dm
    nd = dm.sum()
    ns = sm.sum()
    if ge_d:      # derivative: dangerous wants deriv >= 0
        ld = (torch.relu(-v + eps_d) * dm).sum() / (1e-5 + nd)
        ad = ((v >= 0).to(v.dtype) * dm).sum() / (1e-5 + nd)
    else:         # barrier: dangerous wants h <= -eps
        ld = (torch.relu(v + eps_d) * dm).sum() / (1e-5 + nd)
        ad = ((v <= 0).to(v.dtype) * dm).sum() / (1e-5 + nd)
    ls = (torch.relu(-v) * sm).sum() / (1e-5 + ns)
    acs = ((v > 0).to(v.dtype) * sm).sum() / (1e-5 + ns)
    neg = torch.tensor(-1.0, dtype=v.dtype, device=v.device)
    ad = torch.where(nd > 0, ad, neg)
    acs = torch.where(ns > 0, acs, neg)
    return ld, ls, ad, acs


def loss_barrier(h, states):
    """(loss_dang, loss_safe, acc_dang, acc_safe) (core.py:89-129). h: (N,1,K) or (N,K)."""
    dang = ttc_dangerous_mask(states)[..., 0]
    return _masked_terms(_flat_h(h), dang, LOSS_EPS_DANG, ge_d=False)


def loss_derivatives(states, actions, h, cbf):
    """Discrete CBF condition h(s') - h(s) + dt*alpha*h(s) >= 0 (core.py:132-171).

    h' is evaluated on the time-t neighbour set (defect D10, reuse_nbr_idx).
    """
    s_next = states + dynamics(states, actions) * TIME_STEP
    idx = _knn(states)
    h_next = _flat_h(cbf(s_next, idx=idx.unsqueeze(0)))
    deriv = h_next - _flat_h(h) + TIME_STEP * ALPHA_CBF * _flat_h(h)
    dang = ttc_dangerous_mask(states)[..., 0]
    return _masked_terms(deriv, dang, LOSS_EPS_DANG, ge_d=True)


def loss_actions(s, g, a):
    """mean |‖a‖² − ‖a_ref‖²| with the LQR-like K_ref (core.py:174-184)."""
    return _O.action_loss_terms(s, g, a).mean()
