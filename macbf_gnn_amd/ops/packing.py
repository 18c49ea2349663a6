"""Packing of ONE network's parameters (a standalone ``nn.Module``) into the kernels' layouts.

The training engine packs from the trainer's flat master buffer (``ops.weights``); the
reference-compatible modules (``models.CBF`` / ``models.Controller`` used directly, e.g. by
``core.loss_derivatives`` or an evaluation script) own ordinary parameters. This module builds
the same index tables against the offsets of ``torch.cat(module.parameters())`` and caches them
per (architecture, device); a forward call costs one concat + a few gathers (~50 k elements).
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch

from . import layout as L

_CACHE: Dict[Tuple[str, str], "ModulePack"] = {}


def _offsets(module):
    offs, shapes, o = {}, [], 0
    for name, p in module.named_parameters():
        offs[name] = o
        shapes.append((name, tuple(p.shape), o, p.numel()))
        o += p.numel()
    return offs, shapes, o


DTYPE_PREC = {torch.bfloat16: "bf16", torch.float16: "fp16", torch.float32: "fp32"}


def gather16(src: torch.Tensor, idx: torch.Tensor, dtype, x3: bool) -> torch.Tensor:
    """out[i] = h16(src[idx[i]]); x3: entries flagged with layout.LO_FLAG get the bf16 residual
    src - bf16(src) (the lo plane). Host / module-API twin of the pack_gather kernel."""
    if not x3:
        return src.index_select(0, idx).to(dtype)
    v = src.index_select(0, idx & (L.LO_FLAG - 1))
    hi = v.to(torch.bfloat16)
    lo = (v - hi.float()).to(torch.bfloat16)
    return torch.where((idx & L.LO_FLAG) != 0, lo, hi)


class ModulePack:
    def __init__(self, kind: str, module, device, dtype=torch.float32):
        self.kind = kind
        self.prec = DTYPE_PREC[dtype]     # bf16 | fp16 | fp32 (x3 split kernels)
        self.x3 = self.prec == "fp32"
        self.dtype = torch.float16 if self.prec == "fp16" else torch.bfloat16   # packed element type
        offs, self.shapes, self.n = _offsets(module)
        dim = module.in_dim // 2
        self.dim = dim
        mk = lambda a: torch.as_tensor(L.resolve(a, self.n), dtype=torch.long, device=device)
        mkl = lambda a: torch.as_tensor(a, dtype=torch.long, device=device)
        if kind == "cbf":
            pk = L.cbf_packer(offs, dim)
            vec, _ = L.cbf_vec_index(offs)
            rm = L.cbf_rm(offs)
            self.maps = {"cbf": tuple(mkl(x) for x in L.cbf_grad_map(offs, dim))}
        elif kind == "ctrl":
            pk = L.ctrl_packer(offs, dim)
            vec, _ = L.ctrl_vec_index(offs, dim)
            rm = L.ctrl_node_rm(offs, dim)
            self.maps = {"node": tuple(mkl(x) for x in L.ctrl_node_grad_map(offs, dim)),
                         "edge": tuple(mkl(x) for x in L.ctrl_edge_grad_map(offs, dim))}
        else:
            raise ValueError(kind)
        self.off = pk.offsets()
        self.rm_off = rm.offsets()
        iw, irm = L.resolve(pk.index(), self.n), L.resolve(rm.index(), self.n)
        if self.x3:
            iw, irm = L.x3_frags(iw), L.x3_planes(irm)
        self._iw, self._iv, self._irm = mkl(iw), mk(vec), mkl(irm)
        self._const = torch.tensor([0.0, 1.0], dtype=torch.float32, device=device)

    @torch.no_grad()
    def pack(self, params):
        src = torch.cat([p.detach().float().reshape(-1) for p in params] + [self._const])
        w = gather16(src, self._iw, self.dtype, self.x3)
        v = src.index_select(0, self._iv).contiguous()
        rm = gather16(src, self._irm, self.dtype, self.x3)
        return w, v, rm

    def unpack_grads(self, reds: Dict[str, torch.Tensor]):
        """Per-network slab reductions -> list of per-parameter gradient tensors."""
        flat = torch.zeros(self.n, dtype=torch.float32, device=next(iter(reds.values())).device)
        for name, red in reds.items():
            s, d = self.maps[name]
            flat.index_add_(0, d, red.index_select(0, s))
        return [flat[o:o + n].view(shape) for (_, shape, o, n) in self.shapes]


def module_pack(kind: str, module, device, dtype=None) -> ModulePack:
    """``dtype`` defaults to the module's ``mfma_dtype`` attribute: torch.float32 (unset: the
    reference precision, fp32-accurate x3 kernels), torch.bfloat16 or torch.float16 (one 16-bit
    MFMA per product)."""
    dtype = dtype or getattr(module, "mfma_dtype", torch.float32)
    key = (kind, module.in_dim, str(device), dtype)
    mp = _CACHE.get(key)
    if mp is None:
        mp = ModulePack(kind, module, device, dtype)
        _CACHE[key] = mp
    return mp
