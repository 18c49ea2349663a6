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

``MACBF_DP_FORCE_PG=1`` initialises the process group even at world size 1, so every collective
of a single-GPU run really goes through RCCL on the HIP stream (the RCCL-path test at world 1,
tests/test_gpu_dp.py); with the default, world 1 short-circuits every collective.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


def env_world():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class DP:
    """Thin data-parallel context. ``world == 1`` makes every collective a no-op."""

    def __init__(self, backend: str | None = None, device: torch.device | None = None):
        self.world, self.rank, self.local_rank = env_world()
        self.device = device
        self.owns_pg = False
        self.forced = os.environ.get("MACBF_DP_FORCE_PG", "0") == "1"
        if (self.world > 1 or self.forced) and not dist.is_initialized():
            if self.world == 1:      # a standalone single-process group (no launcher)
                os.environ.setdefault("RANK", "0")
                os.environ.setdefault("WORLD_SIZE", "1")
                os.environ.setdefault("MASTER_PORT", str(_free_port()))
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
        return self.world > 1 or (self.forced and dist.is_initialized())

    @property
    def backend(self) -> str | None:
        return dist.get_backend() if dist.is_initialized() else None

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

    def gather_ints(self, vals: list[int]) -> list[tuple]:
        """Every rank's `vals` (same length on all ranks), ordered by rank: one SUM all-reduce of a
        (world, len) int64 table in which each rank fills its own row (no object pickling)."""
        if not self.enabled:
            return [tuple(int(v) for v in vals)]
        dev = self.device if (dist.get_backend() == "nccl" and self.device is not None) else "cpu"
        t = torch.zeros(self.world, len(vals), dtype=torch.int64, device=dev)
        t[self.rank] = torch.tensor([int(v) for v in vals], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return [tuple(r) for r in t.cpu().tolist()]

    def shutdown(self):
        if self.owns_pg and dist.is_initialized():
            dist.destroy_process_group()
