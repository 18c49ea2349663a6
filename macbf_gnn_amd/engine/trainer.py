"""The training driver: models, flat params, Adam, DP, scenario sampling, logging, ckpt.

Reference: ``train.py:26-105`` (one env, one process, host scenario sampling, two Adams,
tqdm, no logging/ckpt). Here one ``train_step`` is::

    sample B envs (rank-sharded, counter-based RNG)      -> s0 (B,N,4), g (B,N,2)
    engine.step(s0, g)  # rollout + losses + grads into the flat grad buffer
    DP all-reduce(flat grad)                              (one RCCL call)
    Adam on the controller / CBF ranges                   (joint, or alternating)
    engine.after_update()                                 (repack bf16 MFMA fragments)

``engine`` is the HIP engine on a GPU (native kernels, no autograd) or the pure-torch
oracle engine on CPU.
"""
from __future__ import annotations

import os

import time
from typing import Optional

import numpy as np
import torch

from .. import config as C
from .. import env as E
from ..models import CBF, Controller
from ..parallel import DP
from ..utils.params import FlatParams, FlatAdam
from ..utils.metrics import MetricsLogger
from ..utils.timing import PhaseTimer
from ..utils import ckpt


def resolve_device(name: str, local_rank: int = 0) -> torch.device:
    if name in ("auto", None):
        name = "hip" if torch.cuda.is_available() else "cpu"
    if name in ("hip", "cuda", "gpu"):
        if not torch.cuda.is_available():
            raise RuntimeError("HIP device requested but torch.cuda.is_available() is False")
        return torch.device("cuda", local_rank % max(torch.cuda.device_count(), 1))
    return torch.device("cpu")


class Trainer:
    def __init__(self, cfg: C.TrainConfig, device: Optional[torch.device] = None, dp: Optional[DP] = None):
        self.cfg = cfg
        if dp is None:
            from ..parallel import env_world
            _, _, lr_ = env_world()
            device = device or resolve_device(cfg.device, lr_)
            if device.type == "cuda":
                torch.cuda.set_device(device)
            dp = DP(device=device)
        self.dp = dp
        self.device = device or resolve_device(cfg.device, dp.local_rank)
        torch.manual_seed(cfg.seed)
        if cfg.dim not in (2, 3):
            raise ValueError("dim must be 2 or 3")
        self.controller = Controller(2 * cfg.dim).to(self.device)
        self.cbf = CBF(2 * cfg.dim).to(self.device)
        self.fp = FlatParams({"controller": self.controller, "cbf": self.cbf}, device=self.device)
        dp.broadcast_(self.fp.flat)
        self.opt = FlatAdam(self.fp, lr=cfg.lr, weight_decay=cfg.weight_decay)
        self.step_count = 0
        self.torch_gen = torch.Generator(device=self.device)
        self.torch_gen.manual_seed(cfg.seed * 1000003 + dp.rank)
        self.logger = MetricsLogger(dp, cfg.log_path)
        self.timer = PhaseTimer(self.device, enabled=cfg.phase_timing)
        self._host_skipped = 0
        # fp16 mixed precision: dynamic loss scaling. The scale multiplies the
        # in-kernel upstream gradients and is divided out of the flat gradient before the
        # all-reduce; a non-finite step is skipped and halves it.
        self.fp16 = cfg.dtype == "fp16" and self.device.type == "cuda"
        # on the device (fp16): the scale and the finite-step count live in device memory and are
        # updated by the optimizer's commit kernel -- no host round trip per step
        self.gscale_dev = None
        self._grad_scale = float(cfg.loss_scale_init) if self.fp16 else 1.0
        if self.fp16:
            self.gscale_dev = torch.full((1,), float(cfg.loss_scale_init), dtype=torch.float32, device=self.device)
            self._good_dev = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._next = None
        # the next iteration's scenarios on a side stream, launched as soon as enqueued: it runs in
        # the idle issue slots of the current iteration's CBF backward (inline sampling and a side
        # stream gated on the enqueued work both measured slower, docs/PERF.md round 5)
        self._side = (torch.cuda.Stream(device=self.device)
                      if (self.device.type == "cuda" and cfg.prefetch_data) else None)
        # (the sampler's arrays in global memory -- no LDS, so it would share CUs with the kernels it
        # overlaps -- measured much slower: headline 12.10 vs 10.23-10.28 ms, profiles/r6_runs/r6l/)
        if self.device.type == "cuda":
            from .hip_engine import HipEngine
            self._ok = torch.ones(1, dtype=torch.int32, device=self.device)
            self.engine = HipEngine(self)
            if (cfg.nan_guard or self.fp16) and not self.dp.enabled:
                self.engine.check_ok = self._ok      # the finite check runs in the assembly launch
        else:
            from .oracle_engine import OracleEngine
            self.engine = OracleEngine(self)
        if cfg.model_path and _exists(cfg.model_path):
            ckpt.load(self, cfg.model_path)

    # ------------------------------------------------------------------ data
    def sample(self, it: Optional[int] = None):
        """B scenarios for this rank -> (s0, g, obstacles or None): the parallel RSA sampler, on
        the device (HIP kernel) or in the host runtime (C++), identical for one seed."""
        it = self.step_count if it is None else it
        cfg = self.cfg
        B, N = cfg.num_envs, cfg.num_agents
        from ..ops import scenario
        return scenario.generate(B, N, seed=cfg.seed, iteration=it, rank=self.dp.rank, device=self.device,
                                 dim=cfg.dim, num_obstacles=cfg.num_obstacles, obstacle_points=cfg.obstacle_points)

    def _sample_async(self, it: int):
        """Launch the (parameter-independent) scenario sampler for iteration ``it`` on a side
        stream: it overlaps the current iteration's rollout instead of serialising with it."""
        with torch.cuda.stream(self._side):
            data = self.sample(it)
            ev = torch.cuda.Event()
            ev.record(self._side)
        return it, data, ev

    def _take_sample(self):
        if self._side is None:
            return self.sample()
        nx = self._next
        if nx is not None and nx[0] == self.step_count:
            _, data, ev = nx
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            for t in data:
                if t is not None:
                    t.record_stream(cur)
        else:
            data = self.sample()
        self._next = self._sample_async(self.step_count + 1)
        return data

    @property
    def grad_scale(self) -> float:
        """Current loss scale of the upstream gradients (fp16: read from the device)."""
        if self.gscale_dev is not None:
            return float(self.gscale_dev.item())
        return self._grad_scale

    @grad_scale.setter
    def grad_scale(self, v):
        if self.gscale_dev is not None:
            self.gscale_dev.fill_(float(v))
            self._good_dev.zero_()
        else:
            self._grad_scale = float(v)

    def on_params_loaded(self):
        self.fp.rebind()
        self.engine.after_update()

    # ------------------------------------------------------------------ step
    def groups_to_step(self):
        k = self.cfg.alternate_every
        if k <= 0:
            return ["controller", "cbf"]
        return ["controller"] if (self.step_count // k) % 2 == 0 else ["cbf"]

    def train_step(self, s0=None, g=None, obs=None):
        tm = self.timer
        tm.start()
        if s0 is None:
            s0, g, obs = self._take_sample()
        s0 = s0.to(self.device)
        g = g.to(self.device)
        obs = obs.to(self.device) if obs is not None else None
        tm.mark("sample")
        stats = self.engine.step(s0, g, obs)
        self.reduce_grad()
        tm.mark("allreduce")
        # failure detection: a non-finite reduced gradient is identical on every
        # rank, so every rank skips the same step; parameters and Adam state stay untouched
        if self.device.type == "cuda":
            # on the device: grad_check clears a flag that gates the fused Adam kernels; the commit
            # kernel counts the step (or the skip), updates the fp16 loss scale, writes both into
            # this step's statistics row and re-arms the flag -- no host round trip, no torch glue
            from ..ops import native
            guard = self.cfg.nan_guard or self.fp16
            if guard and getattr(self.engine, "check_ok", None) is None:
                native.grad_check(self.fp.grad, self._ok)        # after the all-reduce (DP)
            row = getattr(stats, "row", None)
            row = row if (row is not None and row.numel() >= 18) else None
            # without a stats row the skip flag is read before the commit kernel re-arms it
            ok_snap = self._ok.clone() if (row is None and guard) else None
            # a graph-replayed backward leaves the row's values in its fixed buffer: the commit copies
            take = getattr(self.engine, "take_stats_src", None)
            src = take(row) if (take is not None and row is not None) else None
            # Adam of every group in one launch; its commit (step counts, skip count, loss scale,
            # flag re-arm) runs inside the weight repack launch that follows
            commit = self.opt.step(self.groups_to_step(), ok=self._ok if guard else None, gscale=self.gscale_dev,
                                   good=self._good_dev if self.fp16 else None, growth=self.cfg.loss_scale_growth,
                                   stats_row=row, defer_commit=True, stats_src=src)
            self.engine.after_update(commit=commit)
            if row is None:
                stats["skipped"] = 1 - ok_snap[0] if ok_snap is not None else 0
            elif self.fp16:
                stats.scaled = True
        elif self.cfg.nan_guard and not bool(torch.isfinite(self.fp.grad).all()):
            self._host_skipped += 1
            stats["skipped"] = 1
            if self.dp.rank == 0:
                print(f"[macbf] step {self.step_count}: non-finite gradient, optimizer step skipped "
                      f"({self.skipped_steps} so far)", flush=True)
        else:
            self.opt.step(self.groups_to_step())
            self.engine.after_update()
        tm.mark("optimizer")
        self.step_count += 1
        if tm.enabled:
            stats["phases_ms"] = tm.results()
        return stats

    def reduce_grad(self):
        """DP all-reduce of the flat gradient of the last engine.step (the HIP engine overlaps the
        CBF range with its BPTT and joins it here)."""
        red = getattr(self.engine, "reduce_grad", None)
        if red is not None:
            red()
        else:
            self.dp.all_reduce_(self.fp.grad)

    @property
    def skipped_steps(self) -> int:
        """Optimizer steps skipped by the failure guard (host path + device-side guard)."""
        n = self._host_skipped
        if getattr(self.opt, "on_device", False):
            n += int(self.opt.dskipped.item())
        return n

    def fit(self, steps: Optional[int] = None, progress: bool = False):
        """Train ``steps`` iterations; by default up to ``cfg.train_steps`` in total, so a run
        resumed from a checkpoint continues where it stopped (TRAIN_STEPS, train.py:48)."""
        steps = max(0, self.cfg.train_steps - self.step_count) if steps is None else steps
        it = range(steps)
        if progress and self.dp.rank == 0:
            try:
                from tqdm import tqdm
                it = tqdm(it)
            except ImportError:
                pass
        last = None
        for _ in it:
            stats = self.train_step()
            self.logger.update(stats)
            if (self.step_count % max(self.cfg.display_steps, 1)) == 0:
                last = self.logger.emit(self.step_count)
            if self.cfg.model_path and (self.step_count % max(self.cfg.save_steps, 1)) == 0:
                ckpt.save(self, self.cfg.model_path)
                self.dp.barrier()
        if self.cfg.model_path and steps > 0 and (self.step_count % max(self.cfg.save_steps, 1)) != 0:
            ckpt.save(self, self.cfg.model_path)      # final state of the run
            self.dp.barrier()
        return last

    def save(self, path):
        ckpt.save(self, path)


def _exists(p):
    import os
    return os.path.exists(p)
