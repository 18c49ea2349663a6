"""Per-phase timing of a training iteration.

``PhaseTimer.mark(name)`` closes the phase that started at the previous mark. On a HIP
device the marks are stream events (no host sync until ``results()``), so enabling the
timer does not perturb the pipelined rollout; on CPU they are ``perf_counter`` stamps.
"""
from __future__ import annotations

import time
from typing import Dict, List, Tuple

import torch


class PhaseTimer:
    def __init__(self, device: torch.device, enabled: bool = True):
        self.enabled = enabled
        self.cuda = device.type == "cuda"
        self.marks: List[Tuple[str, object]] = []

    def start(self):
        self.marks = []
        self._stamp("__start__")

    def _stamp(self, name):
        if not self.enabled:
            return
        if self.cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self.marks.append((name, ev))
        else:
            self.marks.append((name, time.perf_counter()))

    def mark(self, name: str):
        self._stamp(name)

    def results(self) -> Dict[str, float]:
        """Milliseconds per phase (syncs the device once)."""
        if not self.enabled or len(self.marks) < 2:
            return {}
        out: Dict[str, float] = {}
        if self.cuda:
            self.marks[-1][1].synchronize()
        for (_, a), (name, b) in zip(self.marks[:-1], self.marks[1:]):
            ms = a.elapsed_time(b) if self.cuda else (b - a) * 1000.0
            out[name] = out.get(name, 0.0) + ms
        return out
