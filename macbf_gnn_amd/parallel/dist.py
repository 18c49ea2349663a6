"""Batched-environment data parallelism over ``torch.distributed``.

One process per GPU; backend ``nccl`` (= RCCL on ROCm, intra-node over xGMI) on HIP
devices, ``gloo`` on CPU. The reference has no parallelism; the collectives of
this framework are exactly:

1. ``all_reduce(SUM)`` of the per-rank loss *counts* (n_dang, n_safe, n_act) right after the
   rollout, so every rank normalises with the global pooled counts and the summed
   gradient equals the single-process gradient on the concatenated env batch;
2. ``all_reduce(SUM)`` of the ONE flat fp32 gradient bucket (51,141 floats = 204.6 KB):
   a latency-bound message on xGMI, so it is issued as a single call (no bucketing);
3. ``broadcast`` of the initial flat parameters from rank 0 (once);
4. ``all_reduce(SUM)`` of a small metrics vector at display steps.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


def env_world():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), \
        int(os.environ.get("LOCAL_RANK", "0"))


class DP:
    """Thin data-parallel context. ``world == 1`` makes every collective a no-op."""

    def __init__(self, backend: str | None = None, device: torch.device | None = None):
        self.world, self.rank, self.local_rank = env_world()
        self.device = device
        self.owns_pg = False
        if self.world > 1 and not dist.is_initialized():
            if backend is None:
                # MACBF_DP_BACKEND=gloo rehearses multi-rank runs with several ranks sharing one
                # GPU (RCCL places one rank per device)
                backend = os.environ.get("MACBF_DP_BACKEND") or (
                    "nccl" if (device is not None and device.type == "cuda") else "gloo")
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            kw = {}
            if backend == "nccl" and device is not None:
                kw["device_id"] = device
            dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=600), **kw)
            self.owns_pg = True
        if dist.is_initialized():
            self.world = dist.get_world_size()
            self.rank = dist.get_rank()

    @property
    def enabled(self):
        return self.world > 1

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.enabled:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t

    def all_reduce_async(self, t: torch.Tensor):
        if self.enabled:
            return dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True)
        return None

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.enabled:
            dist.broadcast(t, src=src)
        return t

    def barrier(self):
        if self.enabled:
            if dist.get_backend() == "nccl" and self.device is not None:
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def max_scalar(self, x: float) -> float:
        if not self.enabled:
            return x
        t = torch.tensor([x], dtype=torch.float64,
                         device=self.device if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def shutdown(self):
        if self.owns_pg and dist.is_initialized():
            dist.destroy_process_group()
