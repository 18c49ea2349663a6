"""Flat fp32 parameter / gradient buffers and a flat Adam.

All 51,141 trainable parameters (controller 34,052 + CBF 17,089) live in ONE
contiguous fp32 buffer; the ``nn.Module`` parameters are views into it, so ``state_dict``
keeps the reference keys while the native kernels, the single RCCL all-reduce and the fused
Adam all work on one flat tensor (one 204.6 KB bucket, no DDP hooks).

The two reference optimizers (``train.py:36-37``: Adam(lr=1e-4, weight_decay=1e-8) on the
controller and on the CBF) are one flat Adam over two contiguous ranges with their own
step counters; the math is ``torch.optim.Adam`` (L2 weight decay added to the gradient).
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch
import torch.nn as nn


class FlatParams:
    """Owns the flat master buffer; module parameters become views into it."""

    def __init__(self, modules: Dict[str, nn.Module], device=None):
        self.modules = modules
        self.specs: List[Tuple[str, str, torch.Size, int, int]] = []
        self.ranges: Dict[str, Tuple[int, int]] = {}
        off = 0
        for mname, mod in modules.items():
            start = off
            for pname, p in mod.named_parameters():
                self.specs.append((mname, pname, p.shape, off, p.numel()))
                off += p.numel()
            self.ranges[mname] = (start, off)
        self.numel = off
        dev = device if device is not None else next(iter(modules.values())).parameters().__next__().device
        self.flat = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        self.grad = torch.zeros_like(self.flat)
        with torch.no_grad():
            for (mname, pname, shape, o, n), p in zip(self.specs, self._params()):
                self.flat[o:o + n].copy_(p.detach().reshape(-1))
        self.rebind()

    def _params(self):
        for mod in self.modules.values():
            for _, p in mod.named_parameters():
                yield p

    def rebind(self):
        """(Re)point every module parameter and its .grad at views of the flat buffers."""
        for (mname, pname, shape, o, n), p in zip(self.specs, self._params()):
            p.data = self.flat[o:o + n].view(shape)
            p.grad = self.grad[o:o + n].view(shape)

    def offset(self, mname: str, pname: str) -> int:
        for m, pn, shape, o, n in self.specs:
            if m == mname and pn == pname:
                return o
        raise KeyError((mname, pname))

    def view(self, mname: str, pname: str) -> torch.Tensor:
        for m, pn, shape, o, n in self.specs:
            if m == mname and pn == pname:
                return self.flat[o:o + n].view(shape)
        raise KeyError((mname, pname))

    def zero_grad(self):
        self.grad.zero_()
        self.rebind()

    def sync_grads_from_modules(self):
        """Autograd may replace a ``.grad`` view by a fresh tensor; fold those back in."""
        for (mname, pname, shape, o, n), p in zip(self.specs, self._params()):
            gv = self.grad[o:o + n]
            if p.grad is None:
                continue
            if p.grad.data_ptr() != gv.data_ptr():
                gv.copy_(p.grad.reshape(-1))
        self.rebind()


class FlatAdam:
    """torch.optim.Adam semantics over contiguous ranges of a flat buffer.

    ``step(group)`` updates one named range (or all). On a HIP device the update runs in
    the fused ``adam`` kernel (``csrc/adam.hip``); on CPU in torch ops.
    """

    def __init__(self, fp: FlatParams, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        self.fp = fp
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.exp_avg = torch.zeros_like(fp.flat)
        self.exp_avg_sq = torch.zeros_like(fp.flat)
        self._names = list(fp.ranges)
        self.on_device = fp.flat.device.type != "cpu"
        self._steps = {name: 0 for name in fp.ranges}
        if self.on_device:
            # step counters and the skipped-step count live on the device: the fused Adam kernel
            # reads them (bias corrections) and a guard flag, so a step needs no host round trip
            dev = fp.flat.device
            self._dsteps = torch.zeros(len(self._names), dtype=torch.int32, device=dev)
            self.dskipped = torch.zeros(1, dtype=torch.int32, device=dev)
            self._one = torch.ones(1, dtype=torch.int32, device=dev)

    @property
    def steps(self):
        """Per-group step counts (host dict; synchronises with the device counters on HIP)."""
        if self.on_device:
            v = self._dsteps.tolist()
            return {n: int(v[i]) for i, n in enumerate(self._names)}
        return dict(self._steps)

    def set_step(self, name, step):
        if self.on_device:
            self._dsteps[self._names.index(name)] = int(step)
        else:
            self._steps[name] = int(step)

    def step(self, groups=None, ok=None, gscale=None, good=None, growth=1000, stats_row=None, defer_commit=False,
             stats_src=None):
        """One Adam step of the named ranges. On HIP, ok (device int32 flag, optional) gates the
        whole step on the device: 0 leaves parameters, moments and step counts untouched and
        counts a skipped step; the commit kernel then re-arms the flag. gscale / good (fp16): the
        device loss scale and finite-step count, updated by the commit kernel (``native.step_commit``);
        stats_row: the iteration's statistics row (skipped flag and loss scale written into it;
        stats_src: its first 16 values are copied from there first).
        All groups update in ONE launch; defer_commit: return the commit's arguments instead of
        launching it (the weight repack runs it: ``PackedWeights.update(commit=...)``)."""
        groups = list(self.fp.ranges) if groups is None else list(groups)
        if self.on_device:
            from ..ops import native
            flag = self._one if ok is None else ok
            mask, spec = 0, []
            for name in groups:
                a, b = self.fp.ranges[name]
                gi = self._names.index(name)
                spec.append((a, b, self._dsteps[gi:gi + 1]))
                mask |= 1 << gi
            if spec:
                native.adam_multi(self.fp.flat, self.fp.grad, self.exp_avg, self.exp_avg_sq, spec, self.lr,
                                  self.betas[0], self.betas[1], self.eps, self.wd, ok=flag)
            kw = dict(gscale=gscale, good=good, growth=growth, stats_row=stats_row, stats_src=stats_src)
            if defer_commit:
                return native.step_commit_args(flag, self._dsteps, mask, self.dskipped, **kw)
            native.step_commit(flag, self._dsteps, mask, self.dskipped, **kw)
            return None
        for name in groups:
            a, b = self.fp.ranges[name]
            self._steps[name] += 1
            self._step_torch(a, b, self._steps[name])

    def _step_torch(self, a, b, t):
        b1, b2 = self.betas
        p = self.fp.flat[a:b]
        g = self.fp.grad[a:b]
        if self.wd != 0:
            g = g + self.wd * p
        m = self.exp_avg[a:b]
        v = self.exp_avg_sq[a:b]
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1 = 1 - b1 ** t
        bc2 = 1 - b2 ** t
        denom = (v.sqrt() / (bc2 ** 0.5)).add_(self.eps)
        p.addcdiv_(m, denom, value=-self.lr / bc1)

    # -- torch.optim.Adam-compatible state dicts (one per reference optimizer) ------------
    def torch_state_dict(self, name: str) -> dict:
        a, _ = self.fp.ranges[name]
        state, ids = {}, []
        i = 0
        nstep = self.steps[name]
        for m, pn, shape, o, n in self.fp.specs:
            if m != name:
                continue
            if nstep > 0:
                state[i] = {"step": torch.tensor(float(nstep)),
                            "exp_avg": self.exp_avg[o:o + n].view(shape).detach().cpu().clone(),
                            "exp_avg_sq": self.exp_avg_sq[o:o + n].view(shape).detach().cpu().clone()}
            ids.append(i)
            i += 1
        group = {"lr": self.lr, "betas": self.betas, "eps": self.eps, "weight_decay": self.wd,
                 "amsgrad": False, "maximize": False, "foreach": None, "capturable": False,
                 "differentiable": False, "fused": None, "decoupled_weight_decay": False,
                 "params": ids}
        return {"state": state, "param_groups": [group]}

    def load_torch_state_dict(self, name: str, sd: dict):
        i = 0
        step = 0
        for m, pn, shape, o, n in self.fp.specs:
            if m != name:
                continue
            st = sd["state"].get(i, sd["state"].get(str(i)))
            if st is not None:
                self.exp_avg[o:o + n].copy_(st["exp_avg"].reshape(-1))
                self.exp_avg_sq[o:o + n].copy_(st["exp_avg_sq"].reshape(-1))
                step = int(float(st["step"]))
            i += 1
        self.set_step(name, step)
