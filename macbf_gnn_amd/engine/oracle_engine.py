"""Training-step engine on the pure-torch oracle (CPU reference path, BASELINE config #1).

Autograd does the backward (BPTT through the rollout, as ``train.py:58-103``). The HIP
engine (``hip_engine.py``) implements the same step with native kernels and a hand-written
reverse-time recursion; ``tests/`` checks the two against each other.
"""
from __future__ import annotations

import torch

from .. import config as C
from .. import oracle


class OracleEngine:
    name = "oracle"

    def __init__(self, trainer):
        self.tr = trainer

    def after_update(self, commit=None):
        if commit is not None:          # a trainer on a HIP device: the deferred optimizer commit
            from ..ops import native
            native.step_commit_raw(commit)

    def step(self, s0, g, obs=None, forced=None):
        """``forced``: replay a trajectory (``oracle.rollout``), e.g. ``HipEngine.trajectory()``."""
        tr = self.tr
        cfg = tr.cfg
        cp = tr.controller.params_dict()
        bp = tr.cbf.params_dict()
        traj = oracle.rollout(cp, s0, g, top_k=cfg.top_k, inner_loops=cfg.inner_loops,
                              bptt=cfg.bptt, early_stop=cfg.early_stop,
                              noise_prob=cfg.add_noise_prob, noise_scale=cfg.noise_scale,
                              generator=tr.torch_gen, compute_safety=cfg.compute_safety, obs=obs,
                              forced=forced)
        tr.timer.mark("rollout")
        T = traj["A"].shape[1]
        valid = traj["valid"]
        s_d = traj["S"][:, :T].detach()
        dang = oracle.ttc_mask_knn(s_d, traj["idx"], oracle.with_obstacles(s_d, obs))
        vmask = valid[..., None, None]
        N = s0.shape[1]
        counts = torch.stack([(dang & vmask).sum(), (~dang & vmask).sum(),
                              valid.sum() * N]).to(torch.float64)
        tr.dp.all_reduce_(counts)
        ncounts = {"n_dang": float(counts[0]), "n_safe": float(counts[1]), "n_act": float(counts[2])}
        losses, sums, act_sum = oracle.train_losses(cp, bp, traj, g, n_counts=ncounts,
                                                    reuse_nbr_idx=cfg.reuse_nbr_idx, top_k=cfg.top_k, obs=obs)
        tr.timer.mark("losses")
        tr.fp.zero_grad()
        losses["total"].backward()
        tr.fp.sync_grads_from_modules()
        tr.timer.mark("backward")
        agent_steps = int(valid.sum().item()) * N
        safe = float((traj["safe"].to(torch.float64) * valid).sum().item()) if "safe" in traj else 0.0
        stats = {
            "loss_total": float(losses["total"].detach()),
            "loss_dang": float(losses["loss_dang"].detach()), "loss_safe": float(losses["loss_safe"].detach()),
            "loss_dang_deriv": float(losses["loss_dang_deriv"].detach()),
            "loss_safe_deriv": float(losses["loss_safe_deriv"].detach()),
            "loss_action": float(losses["loss_action"].detach()),
            "acc_dang_sum": float(sums["acc_dang"]), "acc_safe_sum": float(sums["acc_safe"]),
            "acc_dang_deriv_sum": float(sums["acc_dang_deriv"]),
            "acc_safe_deriv_sum": float(sums["acc_safe_deriv"]),
            "n_dang": ncounts["n_dang"], "n_safe": ncounts["n_safe"],
            "agent_steps": agent_steps, "safe_agents": safe, "T": T,
        }
        return stats
