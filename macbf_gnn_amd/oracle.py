"""Pure-PyTorch oracle of the *intended* MACBF semantics, batched over environments.

This is the CPU reference path (BASELINE config #1) and the correctness oracle for every
HIP kernel in ``csrc/``. It implements the reference with the fixes of the SURVEY.md
section 2.4 defect register:

* kNN keeps self at slot 0 and always returns indices (D3); K_eff = min(N, TOP_K).
* per-edge features use the (N, K, C) -> per-edge layout, not the channel-scrambling
  reshape (D12); the controller max-pools the *values* (D13).
* the trajectory is a batch of per-timestep graphs (B, T, N, K), not one T*N scene (D14);
  loss means are pooled over all valid (env, t, i, k) entries as in the reference's single
  masked mean.
* h' = CBF(s') on the time-t neighbour set (D10, ``reuse_nbr_idx``).

Shapes: B envs, T steps, N agents, K neighbour slots; state dim 2D = (position D, velocity D)
for the D-dimensional double integrator (D = 2: the reference; D = 3: BASELINE config #5).
Functions accept any leading batch dims ``...`` in front of (N, ·). Static obstacles
 enter as extra non-controlled graph nodes: ``nodes = cat(s, [o, 0])``; agents
are the first N nodes, so agent i is node i and self stays at kNN slot 0.
Reference cites: kNN ``core.py:234-250``; controller ``controller.py:31-63``; CBF
``cbf.py:21-45``; TTC ``core.py:187-231``; losses ``core.py:89-184``; loop ``train.py:48-105``.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F

from . import config as C


# ----------------------------------------------------------------------------- graph
def sdim(s: torch.Tensor) -> int:
    """Spatial dimension D of a (..., 2D) double-integrator state."""
    return s.shape[-1] // 2


def with_obstacles(s: torch.Tensor, obs: Optional[torch.Tensor]) -> torch.Tensor:
    """Graph nodes: the N agents followed by the M static obstacle points (velocity 0)."""
    if obs is None:
        return s
    # obs is (B, M, D) (or (M, D)); s is (B, ..., N, 2D): broadcast over the middle dims
    if obs.dim() == 2:
        obs = obs.unsqueeze(0)
    o = obs.reshape(obs.shape[0], *([1] * (s.dim() - obs.dim())), *obs.shape[1:])
    o = o.expand(*s.shape[:-2], *obs.shape[-2:])
    return torch.cat([s, torch.cat([o.to(s.dtype), torch.zeros_like(o, dtype=s.dtype)], -1)], -2)


def sq_dist(d: torch.Tensor, D: int) -> torch.Tensor:
    """sum_d d_d^2 accumulated in coordinate order (matches the kernels' fp32 order)."""
    out = d[..., 0] * d[..., 0]
    for q in range(1, D):
        out = out + d[..., q] * d[..., q]
    return out


def knn_idx(s: torch.Tensor, k: int, nodes: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Indices (into ``nodes``, default the agents) of the k nearest nodes of every agent,
    nearest first.

    Ties are broken by the lower node index (stable sort); the HIP scan compares (d2, index)
    lexicographically, so it produces the same lists in any candidate order. Self is slot 0
    unless another node sits exactly on it with a lower index.
    """
    nodes = s if nodes is None else nodes
    D = sdim(s)
    d = s[..., :D].unsqueeze(-2) - nodes[..., :D].unsqueeze(-3)      # (..., N, Nn, D): p_i - p_j
    d2 = sq_dist(d, D)
    k = min(k, nodes.shape[-2])
    return torch.sort(d2, dim=-1, stable=True).indices[..., :k]


def gather_nbrs(s: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """s (..., Nn, C) nodes, idx (..., N, K) into them -> s_j (..., N, K, C)."""
    lead = s.shape[:-2]
    Nn, Cc = s.shape[-2:]
    N, K = idx.shape[-2:]
    sf = s.reshape(-1, Nn, Cc)
    ix = idx.reshape(-1, N * K, 1).expand(-1, -1, Cc)
    return torch.gather(sf, 1, ix).reshape(*lead, N, K, Cc)


def edge_rel(s: torch.Tensor, idx: torch.Tensor, nodes: Optional[torch.Tensor] = None):
    """Relative state s_i - s_j (..., N, K, 2D) and the self indicator (..., N, K)."""
    sj = gather_nbrs(s if nodes is None else nodes, idx)
    rel = s.unsqueeze(-2) - sj
    ar = torch.arange(s.shape[-2], device=s.device).view(*([1] * (idx.dim() - 2)), -1, 1)
    eye = (idx == ar).to(s.dtype)
    return rel, eye


# ----------------------------------------------------------------------------- safety
def ttc_dangerous(rel: torch.Tensor, eye: torch.Tensor, r: float, ttc: float) -> torch.Tensor:
    """Time-to-collision danger test on relative states (core.py:187-209 / 212-231).

    Self pairs are shifted to p=(1,..,1) via ``eye`` (core.py:193-194). fp32 throughout.
    """
    D = rel.shape[-1] // 2
    p = [rel[..., q] + eye for q in range(D)]
    v = [rel[..., D + q] for q in range(D)]
    alpha = v[0] * v[0]
    pv = p[0] * v[0]
    pp = p[0] * p[0]
    for q in range(1, D):
        alpha = alpha + v[q] * v[q]
        pv = pv + p[q] * v[q]
        pp = pp + p[q] * p[q]
    beta = 2.0 * pv
    gamma = pp - r * r
    disc = beta * beta - 4.0 * alpha * gamma
    dist_dang = gamma < 0
    two_pos = (disc > 0) & (gamma > 0) & (beta < 0)
    lt = (-beta - 2.0 * alpha * ttc < 0) | ((beta + 2.0 * alpha * ttc) ** 2 < disc)
    return dist_dang | (two_pos & lt)


def ttc_mask_knn(s: torch.Tensor, idx: torch.Tensor, nodes: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Training danger mask on the top-K pairs, r=DIST_MIN_THRES, ttc=TIME_TO_COLLISION."""
    rel, eye = edge_rel(s, idx, nodes)
    return ttc_dangerous(rel, eye, C.DIST_MIN_THRES, C.TIME_TO_COLLISION)


def ttc_mask_all_pairs(s: torch.Tensor, nodes: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Check mask of every agent against every node (core.py:212-231) -> (..., N, Nn) bool."""
    nodes = s if nodes is None else nodes
    rel = s.unsqueeze(-2) - nodes.unsqueeze(-3)
    N, Nn = s.shape[-2], nodes.shape[-2]
    eye = torch.eye(N, Nn, dtype=s.dtype, device=s.device).expand(rel.shape[:-1])
    return ttc_dangerous(rel, eye, C.DIST_MIN_CHECK, C.TIME_TO_COLLISION_CHECK)


def safe_agent_count(s: torch.Tensor, nodes: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Number of agents with no dangerous pair, per leading index (train.py:74-75)."""
    return (~ttc_mask_all_pairs(s, nodes).any(-1)).sum(-1)


# ----------------------------------------------------------------------------- networks
# bf16 kernel emulation (tests only): the bf16 MFMA build rounds at fixed points -- the
# hidden activations entering MFMA layers (not the CBF's fp32 64 -> 1 head), the pooled
# features, and every pre-activation
# gradient dZ (the MFMA input of both dX = W^T dZ and dW = dZ X^T; not the CBF's scalar head)
# plus dL/dpooled. Layer-1
# inputs are exact (hi/lo split along k, csrc/common.h mma_bx) and accumulation is fp32.
# With the weights rounded to bf16 as well, the oracle then evaluates the kernels' function up
# to accumulation order and rounding-boundary ties.
_EMULATE = {"bf16": False}


class emulate_bf16:
    """Context manager: oracle networks round like the bf16 kernels (see above)."""

    def __init__(self, on: bool = True):
        self.on = on

    def __enter__(self):
        self.prev = _EMULATE["bf16"]
        _EMULATE["bf16"] = self.on
        return self

    def __exit__(self, *exc):
        _EMULATE["bf16"] = self.prev


def _round16(x):
    return x.to(torch.bfloat16).to(x.dtype)


class _RoundFwd(torch.autograd.Function):        # activation rounding, straight-through grad
    @staticmethod
    def forward(ctx, x):
        return _round16(x)

    @staticmethod
    def backward(ctx, g):
        return g


class _RoundGrad(torch.autograd.Function):       # identity forward, rounded gradient
    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return _round16(g)


class _HeadBf16(torch.autograd.Function):
    """The CBF's 64 -> 1 head in the bf16 build: fp32 forward and dX = dh w4, but dW4 from
    bf16 dh and bf16 relu(H3) (an MFMA stage, csrc/cbf.hip stage C+D) and db4 = sum of fp32 dh."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        g2 = g.reshape(-1, g.shape[-1])
        dw = _round16(g2).t() @ _round16(x.reshape(-1, x.shape[-1]))
        return g @ w, dw, g2.sum(0)


def _qa(x):
    return _RoundFwd.apply(x) if _EMULATE["bf16"] else x


def _qg(x):
    return _RoundGrad.apply(x) if _EMULATE["bf16"] else x


def _lin(x, w, b, first=False, head=False):
    if w.dim() == 3:          # Conv1d(k=1) weight (out, in, 1)
        w = w[..., 0]
    if head:
        return _HeadBf16.apply(x, w, b) if _EMULATE["bf16"] else F.linear(x, w, b)
    return _qg(F.linear(x if first else _qa(x), w, b))


def controller_forward(p: Dict[str, torch.Tensor], s, g, idx, return_aux=False, nodes=None, pool_slots=None,
                       pool_values=None):
    """Gain-scheduled GNN controller (controller.py:31-63), intended semantics.

    ``p`` is the controller ``state_dict`` (or named parameters) keyed like the reference.
    D-dimensional: edge input [s_i - s_j, eye] (2D+1), node input [pooled, p - g, v] (128+2D),
    2D gains, a_d = -(k_{2d} (p_d - g_d) + k_{2d+1} v_d) (D = 2: the reference law).
    ``pool_slots`` (..., N, 128; 255 = no positive row) replaces the max-pool's argmax by given
    neighbour slots (the kernels' saved argmax): the max-pool subgradient at near-ties is a
    choice, and tests pin it to the kernels' choice (see ``pool_slot_gap``). ``pool_values``
    (tests) replaces the pooled values (straight-through: the gradient is unchanged), e.g. by
    the kernels' stored 16-bit pooled rows, so a rounding-boundary tie of one pooled element
    cannot flip the node MLP's path.
    """
    D = sdim(s)
    rel, eye = edge_rel(s, idx, nodes)
    x = torch.cat([rel, eye.unsqueeze(-1)], dim=-1)                     # (...,N,K,2D+1)
    dist = torch.sqrt(sq_dist(rel, D))
    mask = (dist < C.OBS_RADIUS).to(s.dtype)                            # strict, no eps
    h = F.relu(_lin(x, p["controller_centr_net.0.weight"], p["controller_centr_net.0.bias"], first=True))
    h = F.relu(_lin(h, p["controller_centr_net.2.weight"], p["controller_centr_net.2.bias"]))
    hm = h * mask.unsqueeze(-1)
    if pool_slots is None:
        pooled = hm.max(dim=-2).values                                   # (...,N,128)
    else:
        sl = pool_slots.long()
        has = (sl < hm.shape[-2]).to(hm.dtype)
        pooled = hm.gather(-2, sl.clamp(max=hm.shape[-2] - 1).unsqueeze(-2)).squeeze(-2) * has
    if pool_values is not None:
        pooled = pool_values.to(pooled.dtype) + (pooled - pooled.detach())
    z = torch.cat([_qg(_qa(pooled)), s[..., :D] - g, s[..., D:2 * D]], dim=-1)
    for i, act in ((0, True), (2, True), (4, True), (6, False)):
        z = _lin(z, p[f"controller_dec_net.{i}.weight"], p[f"controller_dec_net.{i}.bias"], first=i == 0)
        if act:
            z = F.relu(z)
    k = 2.0 * torch.sigmoid(z) + 0.2
    a = torch.stack([-(k[..., 2 * q] * (s[..., q] - g[..., q]) + k[..., 2 * q + 1] * s[..., D + q])
                     for q in range(D)], dim=-1)
    if return_aux:
        return a, {"gains": k, "pooled": pooled, "mask": mask, "hm": hm}
    return a


def pool_slot_gap(hm: torch.Tensor, pool_slots: torch.Tensor) -> torch.Tensor:
    """How far given max-pool slots are from the true max: max over (agent, feature) of
    (max_k hm - hm[slot]) / max(max_k hm, tiny) (0 when the slots are argmaxes; 255 = no slot
    must mean no positive row)."""
    top = hm.max(dim=-2).values
    sl = pool_slots.long()
    has = sl < hm.shape[-2]
    val = hm.gather(-2, sl.clamp(max=hm.shape[-2] - 1).unsqueeze(-2)).squeeze(-2)
    gap = torch.where(has, (top - val) / top.clamp_min(1e-30), (top > 0).to(top.dtype))
    return gap.max()


def cbf_features(s, idx, nodes=None):
    D = sdim(s)
    rel, eye = edge_rel(s, idx, nodes)
    d = torch.sqrt(sq_dist(rel, D) + C.CBF_DIST_EPS_COORD * D)
    x = torch.cat([rel, eye.unsqueeze(-1), (d - C.DIST_MIN_THRES).unsqueeze(-1)], dim=-1)
    mask = (d <= C.OBS_RADIUS).to(s.dtype)
    return x, mask


def cbf_forward(p: Dict[str, torch.Tensor], s, idx, nodes=None):
    """Per-edge barrier h(x_i, x_j) (cbf.py:21-45) -> (..., N, K); masked by radius.
    Edge input [s_i - s_j, eye, |p_i - p_j|_eps - r] (2D + 2 channels)."""
    x, mask = cbf_features(s, idx, nodes)
    z = x
    for i, act in ((0, True), (2, True), (4, True), (6, False)):
        # (the 64 -> 1 head is an fp32 dot product on the fp32 relu(H3), csrc/cbf.hip; db4 sums
        # the fp32 dh; dH3 = w4 dh is rounded at layer 3's pre-activation)
        z = _lin(z, p[f"cbf_net.{i}.weight"], p[f"cbf_net.{i}.bias"], first=i == 0, head=i == 6)
        if act:
            z = F.relu(z)
    return z[..., 0] * mask


# ----------------------------------------------------------------------------- losses
def action_ref(s, g):
    """a_ref = [p-g, v] K_ref^T with K_ref = -[I, sqrt3 I] (core.py:175-178; D = 2 there)."""
    D = sdim(s)
    return torch.stack([-((s[..., q] - g[..., q]) + C.SQRT3 * s[..., D + q]) for q in range(D)], dim=-1)


def action_loss_terms(s, g, a):
    """|‖a‖² − ‖a_ref‖²| per agent (core.py:174-184 before the mean)."""
    ar = action_ref(s, g)
    return ((a * a).sum(-1) - (ar * ar).sum(-1)).abs()


def cbf_loss_sums(h, h_next, dang, valid):
    """Raw sums of the 8 barrier/derivative terms + 2 counts (no normalisation).

    h, h_next, dang: (B,T,N,K); valid: (B,T) bool. Returns dict of 0-d tensors.
    """
    w = valid.to(h.dtype)[..., None, None]
    dm = dang.to(h.dtype) * w
    sm = (1.0 - dang.to(h.dtype)) * w
    deriv = h_next - h + C.TIME_STEP * C.ALPHA_CBF * h
    return {
        "n_dang": dm.sum(), "n_safe": sm.sum(),
        "loss_dang": (F.relu(h + C.LOSS_EPS_DANG) * dm).sum(),
        "loss_safe": (F.relu(-h) * sm).sum(),
        "acc_dang": ((h <= 0).to(h.dtype) * dm).sum(),
        "acc_safe": ((h > 0).to(h.dtype) * sm).sum(),
        "loss_dang_deriv": (F.relu(-deriv + C.LOSS_EPS_DANG) * dm).sum(),
        "loss_safe_deriv": (F.relu(-deriv) * sm).sum(),
        "acc_dang_deriv": ((deriv >= 0).to(h.dtype) * dm).sum(),
        "acc_safe_deriv": ((deriv > 0).to(h.dtype) * sm).sum(),
    }


def finalize_losses(sums, n_act_sum, n_act):
    """Normalise pooled sums like core.py:113-127 / 155-169 and weight like train.py:93-98."""
    nd = 1e-5 + sums["n_dang"]
    ns = 1e-5 + sums["n_safe"]
    out = {
        "loss_dang": sums["loss_dang"] / nd,
        "loss_safe": sums["loss_safe"] / ns,
        "loss_dang_deriv": sums["loss_dang_deriv"] / nd,
        "loss_safe_deriv": sums["loss_safe_deriv"] / ns,
        "loss_action": n_act_sum / max(float(n_act), 1.0),
    }
    neg = torch.tensor(-1.0, dtype=nd.dtype, device=nd.device)
    has_d = sums["n_dang"] > 0
    has_s = sums["n_safe"] > 0
    out["acc_dang"] = torch.where(has_d, sums["acc_dang"] / nd, neg)
    out["acc_safe"] = torch.where(has_s, sums["acc_safe"] / ns, neg)
    out["acc_dang_deriv"] = torch.where(has_d, sums["acc_dang_deriv"] / nd, neg)
    out["acc_safe_deriv"] = torch.where(has_s, sums["acc_safe_deriv"] / ns, neg)
    w = C.LOSS_WEIGHTS
    out["total"] = C.LOSS_SCALE * (w[0] * out["loss_dang"] + w[1] * out["loss_safe"]
                                   + w[2] * out["loss_dang_deriv"] + w[3] * out["loss_safe_deriv"]
                                   + w[4] * out["loss_action"])
    return out


# ----------------------------------------------------------------------------- rollout
def rollout(ctrl_params, s0, g, *, top_k=C.TOP_K, inner_loops=C.INNER_LOOPS, bptt=True,
            early_stop=True, noise_prob=0.0, noise_scale=C.NOISE_SCALE, generator=None,
            compute_safety=False, obs=None, forced=None):
    """Batched rollout with per-env done masks (train.py:58-81).

    Returns dict with S (B,T+1,N,4), A (B,T,N,2), idx (B,T,N,K), valid (B,T) bool,
    dist (B,T) mean goal distance after each step, safe (B,T) safe-agent counts of s_{t+1}.

    ``forced`` (tests): replay another engine's trajectory -- dict S (B,T+1,N,2D), idx
    (B,T,N,K), optional slots (B,T,N,128) max-pool argmax. The states take the given values
    while their gradients follow this rollout's own expressions (straight-through:
    s_{t+1} = S_{t+1} + (e - e.detach()), e = s_t + dt [v, a]), so the gradient is the oracle's
    gradient along exactly that trajectory, graph and pooling choice.
    """
    B = s0.shape[0]
    s = s0
    active = torch.ones(B, dtype=torch.bool, device=s0.device)
    S, A, I, V, D, SF = [s0], [], [], [], [], []
    dim = sdim(s0)
    if forced is not None:
        inner_loops = forced["idx"].shape[1]
        s = forced["S"][:, 0] + (s0 - s0.detach())
    for t in range(inner_loops):
        nodes = with_obstacles(s, obs)
        if forced is None:
            idx = knn_idx(s.detach(), top_k, nodes.detach())
            a = controller_forward(ctrl_params, s, g, idx, nodes=nodes)
        else:
            idx = forced["idx"][:, t].long()
            sl = forced.get("slots")
            a = controller_forward(ctrl_params, s, g, idx, nodes=nodes, pool_slots=None if sl is None else sl[:, t])
        if noise_prob > 0:
            coin = torch.rand(B, generator=generator, device=s.device) < noise_prob
            nz = torch.randn(a.shape, generator=generator, device=s.device) * noise_scale
            a = a + nz * coin[:, None, None].to(a.dtype)
        s_next = s + torch.cat([s[..., dim:], a], -1) * C.TIME_STEP
        if forced is not None:
            s_next = forced["S"][:, t + 1] + (s_next - s_next.detach())
        dist = torch.linalg.norm(s_next[..., :dim] - g, dim=-1).mean(-1)
        V.append(active.clone())
        A.append(a)
        I.append(idx)
        D.append(dist.detach())
        if compute_safety:
            sn = s_next.detach()
            SF.append(safe_agent_count(sn, with_obstacles(sn, obs)))
        S.append(s_next)
        active = active & ~(dist.detach() < C.DIST_MIN_CHECK)
        s = s_next if bptt else s_next.detach()
        if early_stop and not bool(active.any()):
            break
    out = {"S": torch.stack(S, 1), "A": torch.stack(A, 1), "idx": torch.stack(I, 1),
           "valid": torch.stack(V, 1), "dist": torch.stack(D, 1)}
    if compute_safety:
        out["safe"] = torch.stack(SF, 1)
    if not bptt:
        # keep s_{t+1} connected to a_t for h' but detach s_t inputs (upstream-MACBF mode)
        out["S_in"] = torch.stack([S[0]] + [x.detach() for x in S[1:]], 1)
    return out


def train_losses(ctrl_params, cbf_params, traj, g, *, n_counts: Optional[Dict] = None,
                 reuse_nbr_idx=True, top_k=C.TOP_K, obs=None):
    """All losses of one iteration from a rollout (train.py:83-98, intended semantics).

    ``n_counts`` overrides the pooled counts (n_dang, n_safe, n_act) -- used by DP so that
    every rank normalises by the global counts and the summed gradient equals the
    single-process gradient on the concatenated env batch.
    """
    S, A, idx, valid = traj["S"], traj["A"], traj["idx"], traj["valid"]
    T = A.shape[1]
    S_in = traj.get("S_in", S)
    s_t = S_in[:, :T]
    s_n = S[:, 1:T + 1]
    h = cbf_forward(cbf_params, s_t, idx, nodes=with_obstacles(s_t, obs))
    nodes_n = with_obstacles(s_n, obs)
    idx_n = idx if reuse_nbr_idx else knn_idx(s_n.detach(), top_k, nodes_n.detach())
    hn = cbf_forward(cbf_params, s_n, idx_n, nodes=nodes_n)
    s_d = S[:, :T].detach()
    dang = ttc_mask_knn(s_d, idx, with_obstacles(s_d, obs))
    sums = cbf_loss_sums(h, hn, dang, valid)
    gg = g.unsqueeze(1).expand(-1, T, -1, -1)
    act = action_loss_terms(s_t, gg, A)
    vf = valid.to(act.dtype)[..., None]
    act_sum = (act * vf).sum()
    n_act = float(vf.sum().item()) * S.shape[2]
    if n_counts is not None:
        sums = dict(sums)
        sums["n_dang"] = torch.as_tensor(n_counts["n_dang"], dtype=h.dtype)
        sums["n_safe"] = torch.as_tensor(n_counts["n_safe"], dtype=h.dtype)
        n_act = float(n_counts["n_act"])
    return finalize_losses(sums, act_sum, n_act), sums, act_sum
