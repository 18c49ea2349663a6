"""Evaluation with test-time action refinement (the reference defines
``EVALUATE_STEPS``, ``REFINE_LOOPS``, ``REFINE_LEARNING_RATE`` at ``config.py:17,19-20`` but never
uses them).

Per rollout step:
    idx     = kNN(s_t)                                   (K1, native on the HIP device)
    a       = pi(s_t, g)                                 (controller)
    refine  : a_r = a + delta, delta <- delta - lr * d/d delta  sum_e relu(-(h(s') - h(s) + dt*alpha*h(s)))
              with s' = s + dt * [v, a_r], h on the time-t neighbour slots, until the discrete CBF
              condition holds on every radius-masked edge or REFINE_LOOPS steps are spent
    s_{t+1} = s_t + dt * [v, a_r]
Metrics: safety rate (all-pairs TTC check with DIST_MIN_CHECK / TIME_TO_COLLISION_CHECK, the
``core.py:212-231`` formula), reaching rate (agents within DIST_MIN_CHECK of their goal at the
end), mean final goal distance and refinement statistics.

On a HIP device the CBF and controller run through the native autograd Functions
(``ops/cbf.py``, ``ops/ctrl.py``); on CPU through the fp32 oracle.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

import torch

from . import config as C
from . import oracle


@dataclass
class EvalConfig:
    num_agents: int = 32
    num_envs: int = 1
    episodes: int = C.EVALUATE_STEPS
    max_steps: int = C.INNER_LOOPS
    refine: bool = True
    refine_loops: int = C.REFINE_LOOPS
    refine_lr: float = C.REFINE_LEARNING_RATE
    top_k: int = C.TOP_K
    seed: int = 0
    early_stop: bool = True
    diagnose: bool = False      # dense all-pairs check: are the flagged pairs top-K neighbours?
    refine_space: str = "actions"   # "actions" (upstream MACBF) or "gains": refine only the PD gains
                                    # of the reference controller law (controller.py:53-61) -- what
                                    # the trained policy class itself can express


def _knn(s, k):
    if s.is_cuda:
        from .ops import graph
        return graph.knn(s, k).long()
    return oracle.knn_idx(s, k)


def _safe_count(s):
    if s.is_cuda:
        from .ops import graph
        return graph.safe_agent_count(s)
    return oracle.safe_agent_count(s).float()


def refine_actions(cbf, s, a, idx, loops: int = C.REFINE_LOOPS, lr: float = C.REFINE_LEARNING_RATE,
                   check_every: int = 10):
    """Gradient refinement of the actions on the discrete CBF condition. Returns
    (refined actions, iterations used, remaining violation sum).

    The violation is a hinge: once it is exactly zero its gradient is exactly zero, so further
    iterations leave the actions unchanged. The loop therefore only looks at the violation on
    the host every ``check_every`` iterations (one sync instead of one per iteration); the
    iteration count (iterations that still had a violation) is kept on the device."""
    with torch.no_grad():
        h = cbf(s, idx=idx)
    delta = torch.zeros_like(a, requires_grad=True)
    viol = torch.zeros((), device=s.device)
    used = torch.zeros((), dtype=torch.int64, device=s.device)
    for it in range(1, loops + 1):
        ar = a + delta
        s_next = s + torch.cat([s[..., 2:], ar], -1) * C.TIME_STEP
        hn = cbf(s_next, idx=idx)
        deriv = hn - h + C.TIME_STEP * C.ALPHA_CBF * h
        viol = torch.relu(-deriv).sum()
        pending = viol.detach() > 0
        used += pending.long()
        if it % check_every == 0 and not bool(pending):
            break
        g, = torch.autograd.grad(viol, delta)
        with torch.no_grad():
            delta -= lr * g
    return (a + delta).detach(), int(used), float(viol.detach())


def _pd_action(s, g, y):
    """The reference PD law a_d = -(k_2d (p_d - g_d) + k_2d+1 v_d), k = 2 sigmoid(y) + 0.2."""
    D = s.shape[-1] // 2
    k = 2.0 * torch.sigmoid(y) + 0.2
    return torch.stack([-(k[..., 2 * q] * (s[..., q] - g[..., q]) + k[..., 2 * q + 1] * s[..., D + q])
                        for q in range(D)], dim=-1)


def refine_gains(cbf, s, g, k0, idx, loops: int = C.REFINE_LOOPS, lr: float = C.REFINE_LEARNING_RATE,
                 check_every: int = 10):
    """refine_actions restricted to the controller's action space: gradient steps on the gain
    pre-activations y (k = 2 sigmoid(y) + 0.2, started at the network's gains k0) instead of free
    actions."""
    with torch.no_grad():
        h = cbf(s, idx=idx)
        u = ((k0 - 0.2) / 2.0).clamp(1e-6, 1 - 1e-6)
        y = torch.log(u / (1 - u))
    y = y.clone().requires_grad_(True)
    viol = torch.zeros((), device=s.device)
    used = torch.zeros((), dtype=torch.int64, device=s.device)
    for it in range(1, loops + 1):
        a = _pd_action(s, g, y)
        s_next = s + torch.cat([s[..., 2:], a], -1) * C.TIME_STEP
        hn = cbf(s_next, idx=idx)
        viol = torch.relu(-(hn - h + C.TIME_STEP * C.ALPHA_CBF * h)).sum()
        pending = viol.detach() > 0
        used += pending.long()
        if it % check_every == 0 and not bool(pending):
            break
        gy, = torch.autograd.grad(viol, y)
        with torch.no_grad():
            y -= lr * gy
    with torch.no_grad():
        return _pd_action(s, g, y), int(used), float(viol.detach())


def _unsafe_diag(s_next, idx):
    """(unsafe agents, unsafe agents whose every flagged pair is one of their top-K neighbours at
    the step's graph) -- do the controller / CBF see the pairs that the safety check flags?"""
    dang = oracle.ttc_mask_all_pairs(s_next)                  # (B, N, N) check mask
    unsafe = dang.any(-1)
    in_k = torch.zeros_like(dang)
    in_k.scatter_(-1, idx.long(), True)
    seen = unsafe & ~(dang & ~in_k).any(-1)
    return unsafe.sum(), seen.sum()


def rollout_eval(controller, cbf, s0, g, cfg: EvalConfig) -> Dict[str, float]:
    s = s0
    B, N, _ = s.shape
    k = min(cfg.top_k, N)
    safe_sum = 0.0
    steps = 0
    refine_iters = 0
    unsafe_n = torch.zeros((), device=s.device)
    seen_n = torch.zeros((), device=s.device)
    active = torch.ones(B, dtype=torch.bool, device=s.device)
    for t in range(cfg.max_steps):
        idx = _knn(s, k)
        with torch.no_grad():
            a = controller(s, g, idx=idx)
        if cfg.refine and cfg.refine_space == "gains":
            with torch.no_grad():
                _, aux = oracle.controller_forward(controller.params_dict(), s, g, idx, return_aux=True)
            a, it, _ = refine_gains(cbf, s, g, aux["gains"], idx, cfg.refine_loops, cfg.refine_lr)
            refine_iters += it
        elif cfg.refine:
            a, it, _ = refine_actions(cbf, s, a, idx, cfg.refine_loops, cfg.refine_lr)
            refine_iters += it
        with torch.no_grad():
            s = s + torch.cat([s[..., 2:], a], -1) * C.TIME_STEP
            safe = _safe_count(s)
            safe_sum += float((safe * active.float()).sum())
            if cfg.diagnose:
                u, sn = _unsafe_diag(s[active], idx[active])
                unsafe_n += u
                seen_n += sn
            steps += int(active.sum()) * N
            dist = torch.linalg.vector_norm(s[..., :2] - g, dim=-1).mean(-1)
            active = active & (dist >= C.DIST_MIN_CHECK)
        if cfg.early_stop and not bool(active.any()):
            break
    with torch.no_grad():
        d = torch.linalg.vector_norm(s[..., :2] - g, dim=-1)
        reach = float((d < C.DIST_MIN_CHECK).float().mean())
        mean_dist = float(d.mean())
    out = {"safety_rate": safe_sum / max(steps, 1), "reaching_rate": reach, "mean_goal_dist": mean_dist,
           "steps": t + 1, "agent_steps": steps, "refine_iters": refine_iters}
    if cfg.diagnose:
        out["unsafe_agent_steps"] = float(unsafe_n)
        out["unsafe_pairs_in_topk_share"] = float(seen_n) / max(float(unsafe_n), 1.0)
    return out


def evaluate(controller, cbf, cfg: EvalConfig, device: Optional[torch.device] = None) -> Dict[str, float]:
    """Run ``cfg.episodes`` fresh scenarios; returns metrics averaged over episodes."""
    from . import env as E
    device = device or next(controller.parameters()).device
    controller.eval()
    cbf.eval()
    agg: Dict[str, float] = {}
    for ep in range(cfg.episodes):
        if device.type == "cuda":
            from .ops import scenario
            s0, g, _ = scenario.generate(cfg.num_envs, cfg.num_agents, seed=cfg.seed + 7919, iteration=ep, rank=0,
                                      device=device)
        else:
            s0, g = E.generate_batch(cfg.num_envs, cfg.num_agents, C.DIST_MIN_THRES, seed=cfg.seed * 7919 + ep)
        r = rollout_eval(controller, cbf, s0.to(device), g.to(device), cfg)
        for kk, v in r.items():
            agg[kk] = agg.get(kk, 0.0) + float(v)
    return {kk: v / cfg.episodes for kk, v in agg.items()}
