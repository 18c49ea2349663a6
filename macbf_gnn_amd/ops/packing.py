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


class ModulePack:
    def __init__(self, kind: str, module, device, dtype=torch.bfloat16):
        self.kind = kind
        self.dtype = dtype      # 16-bit MFMA element type (bf16 | fp16)
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
        self._iw, self._iv, self._irm = mk(pk.index()), mk(vec), mk(rm.index())
        self._const = torch.tensor([0.0, 1.0], dtype=torch.float32, device=device)

    @torch.no_grad()
    def pack(self, params):
        src = torch.cat([p.detach().float().reshape(-1) for p in params] + [self._const])
        w = src.index_select(0, self._iw).to(self.dtype)
        v = src.index_select(0, self._iv).contiguous()
        rm = src.index_select(0, self._irm).to(self.dtype)
        return w, v, rm

    def unpack_grads(self, reds: Dict[str, torch.Tensor]):
        """Per-network slab reductions -> list of per-parameter gradient tensors."""
        flat = torch.zeros(self.n, dtype=torch.float32, device=next(iter(reds.values())).device)
        for name, red in reds.items():
            s, d = self.maps[name]
            flat.index_add_(0, d, red.index_select(0, s))
        return [flat[o:o + n].view(shape) for (_, shape, o, n) in self.shapes]


def module_pack(kind: str, module, device, dtype=None) -> ModulePack:
    """``dtype`` defaults to the module's ``mfma_dtype`` attribute (bf16 when unset)."""
    dtype = dtype or getattr(module, "mfma_dtype", torch.bfloat16)
    key = (kind, module.in_dim, str(device), dtype)
    mp = _CACHE.get(key)
    if mp is None:
        mp = ModulePack(kind, module, device, dtype)
        _CACHE[key] = mp
    return mp
