"""Metrics accumulation and JSONL logging.

The reference collects loss/acc lists and never emits them (``train.py:43-45,93-96``) and
has the safety rate commented out (``train.py:74-76``). Here every ``DISPLAY_STEPS`` the
per-rank sums are all-reduced (one small collective) and rank 0 prints one JSON line:
the 5 weighted losses, 4 accuracies, safety rate (fraction of agents with no dangerous
pair under the ``core.py:212-231`` check, averaged over valid steps) and agent-steps/s.
"""
from __future__ import annotations

import collections.abc
import json
import sys
import time

import torch

from .. import config as C

KEYS = ["loss_total", "loss_dang", "loss_safe", "loss_dang_deriv", "loss_safe_deriv", "loss_action",
        "acc_dang_sum", "acc_safe_sum", "acc_dang_deriv_sum", "acc_safe_deriv_sum",
        "n_dang", "n_safe", "agent_steps", "safe_agents", "T", "iters"]
# keys whose per-rank values are already normalised by global counts (sum over ranks);
# n_dang/n_safe are global already (divide by world after the sum)
GLOBAL_KEYS = {"n_dang", "n_safe"}


class StepStats(collections.abc.MutableMapping):
    """Statistics of one training iteration of the HIP engine, kept on the device as ONE raw
    vector (cloned once per iteration) until first read: the derived values (losses,
    accuracies, counts) are then computed on the host from a single device-to-host copy. No
    per-statistic kernels and no host synchronisation inside the training loop.

    raw = [10 loss partial sums (slots 2..9: barrier / derivative hinge sums and accuracy
    counts), n_dang, n_safe, n_act (global pooled counts), agent-steps, safe agents, action-loss
    sum (this rank) (, skipped step, loss scale: written by the optimizer's commit kernel)]."""

    RAW = 16

    def __init__(self, raw: torch.Tensor, T, extra=None):
        self.row = raw               # the device row as written so far (the optimizer's commit completes it)
        self.scaled = False          # fp16: report the loss scale (raw[17])
        self._T = T
        self.extra = dict(extra or {})
        self._host = None
        self.flush = None            # set by a graph-replayed backward: completes the row first

    @property
    def raw(self) -> torch.Tensor:
        """The complete device row (a graph-replayed backward's pending values copied in first)."""
        if self.flush is not None:
            self.flush()
        return self.row

    def _compute(self):
        if self._host is None:
            v = [float(x) for x in self.raw.tolist()]
            sums, (n_dang, n_safe, n_act), (ag, safe, act_sum) = v[:10], v[10:13], v[13:16]
            nd, ns = 1e-5 + n_dang, 1e-5 + n_safe
            w = C.LOSS_WEIGHTS
            d = {"loss_dang": sums[2] / nd, "loss_safe": sums[3] / ns, "loss_dang_deriv": sums[6] / nd,
                 "loss_safe_deriv": sums[7] / ns, "loss_action": act_sum / max(n_act, 1.0),
                 "acc_dang_sum": sums[4], "acc_safe_sum": sums[5], "acc_dang_deriv_sum": sums[8],
                 "acc_safe_deriv_sum": sums[9], "n_dang": n_dang, "n_safe": n_safe,
                 "agent_steps": ag, "safe_agents": safe}
            d["loss_total"] = C.LOSS_SCALE * (w[0] * d["loss_dang"] + w[1] * d["loss_safe"] + w[2] * d["loss_dang_deriv"]
                                              + w[3] * d["loss_safe_deriv"] + w[4] * d["loss_action"])
            d["T"] = float(self._T)
            if len(v) >= 18:
                d["skipped"] = v[16]
                if self.scaled:
                    d["grad_scale"] = v[17]
            for k, x in self.extra.items():
                d[k] = float(x) if isinstance(x, torch.Tensor) else x
            self._host = d
        return self._host

    def __getitem__(self, k):
        return self._compute()[k]

    def __setitem__(self, k, v):
        self.extra[k] = v
        if self._host is not None:
            self._host[k] = float(v) if isinstance(v, torch.Tensor) else v

    def __delitem__(self, k):
        raise KeyError("StepStats entries cannot be deleted")

    def __iter__(self):
        return iter(self._compute())

    def __len__(self):
        return len(self._compute())


class MetricsLogger:
    def __init__(self, dp, path=None, stream=sys.stdout):
        self.dp = dp
        self.path = path
        self.stream = stream
        self.reset()

    def reset(self):
        self.acc = {k: 0.0 for k in KEYS}
        self.pending = []
        self.t0 = time.perf_counter()

    def update(self, stats):
        """Accumulate; device tensors stay on device (no host sync until emit)."""
        if isinstance(stats, StepStats):       # evaluated at emit time
            self.pending.append(stats)
            return
        for k in KEYS:
            if k == "iters":
                self.acc[k] += 1
            elif k in stats:
                v = stats[k]
                if isinstance(v, torch.Tensor):
                    v = v.detach().to(torch.float64)
                self.acc[k] = self.acc[k] + v

    def summary(self, step):
        for st in self.pending:
            for k in KEYS:
                self.acc[k] += 1 if k == "iters" else st[k]
        self.pending = []
        vec = torch.tensor([float(self.acc[k]) for k in KEYS], dtype=torch.float64)
        if self.dp.enabled:
            dev = self.dp.device if (self.dp.device is not None and self.dp.device.type == "cuda") else "cpu"
            vec = vec.to(dev)
            self.dp.all_reduce_(vec)
            vec = vec.cpu()
        d = dict(zip(KEYS, vec.tolist()))
        w = max(self.dp.world, 1)
        it = max(d["iters"] / w, 1.0)
        dt = time.perf_counter() - self.t0
        nd = d["n_dang"] / w
        ns = d["n_safe"] / w
        out = {"step": step, "iters": int(it)}
        for k in ["loss_total", "loss_dang", "loss_safe", "loss_dang_deriv", "loss_safe_deriv", "loss_action"]:
            out[k] = d[k] / it
        out["acc_dang"] = d["acc_dang_sum"] / nd if nd > 0 else -1.0
        out["acc_safe"] = d["acc_safe_sum"] / ns if ns > 0 else -1.0
        out["acc_dang_deriv"] = d["acc_dang_deriv_sum"] / nd if nd > 0 else -1.0
        out["acc_safe_deriv"] = d["acc_safe_deriv_sum"] / ns if ns > 0 else -1.0
        out["safety_rate"] = d["safe_agents"] / d["agent_steps"] if d["agent_steps"] > 0 else 1.0
        out["mean_T"] = d["T"] / (it * w)
        out["agent_steps_per_s"] = d["agent_steps"] / max(dt, 1e-9)
        return out

    def emit(self, step):
        out = self.summary(step)
        if self.dp.rank == 0:
            line = json.dumps(out)
            print(line, file=self.stream, flush=True)
            if self.path:
                with open(self.path, "a") as f:
                    f.write(line + "\n")
        self.reset()
        return out
