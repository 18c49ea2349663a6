"""Per-step repacking of the flat fp32 master parameters into the kernels' bf16 MFMA
fragment buffers (+ fp32 side vectors). One gather per network per optimizer step.

dtype selects the kernel precision (csrc/prec.h): torch.bfloat16 / torch.float16 (one 16-bit
MFMA per product) or torch.float32 -- the fp32-accurate 3-term split kernels, whose packed
buffers (bf16) carry a residual plane next to every fragment / image (layout.x3_*)."""
from __future__ import annotations

import torch

from . import layout as L
from .packing import DTYPE_PREC, gather16


class PackedWeights:
    def __init__(self, fp, dim: int = 2, dtype=torch.bfloat16):
        self.fp = fp
        self.dim = dim
        self.prec = DTYPE_PREC[dtype]                      # bf16 | fp16 | fp32 (x3)
        self.x3 = self.prec == "fp32"
        self.dtype = torch.float16 if self.prec == "fp16" else torch.bfloat16   # packed element type
        offs = {pn: o for (m, pn, shape, o, n) in fp.specs}
        dev = fp.flat.device
        n = fp.numel
        self.ctrl_pk = L.ctrl_packer(offs, dim)
        self.cbf_pk = L.cbf_packer(offs, dim)
        self.ctrl_off = self.ctrl_pk.offsets()
        self.cbf_off = self.cbf_pk.offsets()
        cv, self.ctrl_voff = L.ctrl_vec_index(offs, dim)
        bv, self.cbf_voff = L.cbf_vec_index(offs)
        self.node_rm = L.ctrl_node_rm(offs, dim)
        self.node_rm_off = self.node_rm.offsets()
        self.cbf_rmp = L.cbf_rm(offs)
        # all 16-bit buffers are views of one allocation (segments 256-element aligned), the
        # fp32 side vectors views of another: one gather launch repacks everything
        seg16 = [L.resolve(self.ctrl_pk.index(), n), L.resolve(self.cbf_pk.index(), n),
                 L.resolve(self.node_rm.index(), n), L.resolve(self.cbf_rmp.index(), n)]
        frags = L.x3_frags if self.x3 else (lambda a: a)       # x3: [hi | lo] per fragment
        planes = L.x3_planes if self.x3 else (lambda a: a)     # x3: [hi plane | lo plane] per image
        seg16 = [frags(seg16[0]), frags(seg16[1]), planes(seg16[2]), planes(seg16[3])]
        # the 16x16x32 backward kernels (every precision): CBF (csrc/cbf16.h: permuted W2/W3 images +
        # layer-1 fragments), controller edge (csrc/ctrl16.h) and node (csrc/node16.h)
        self.cbf_rmp16 = L.cbf_rm16(offs)
        self.cbf_pk16 = L.cbf_packer16(offs, dim)
        self.ctrl_pk16 = L.ctrl_edge_packer16(offs, dim)
        self.node_rmp16 = L.node_rm16(offs, dim)
        seg16 += [planes(L.resolve(self.cbf_rmp16.index(), n)),
                  frags(L.resolve(self.cbf_pk16.index(), n)),
                  frags(L.resolve(self.ctrl_pk16.index(), n)),
                  planes(L.resolve(self.node_rmp16.index(), n))]
        seg32 = [L.resolve(cv, n), L.resolve(bv, n)]
        self._idx16, v16 = self._concat(seg16, n, 256)
        self._idx32, v32 = self._concat(seg32, n, 64)
        for a in (self._idx16 & (L.LO_FLAG - 1), self._idx32):   # the gather kernel trusts these bounds
            if a.size and (a.min() < 0 or a.max() > n + 1):
                raise ValueError("packing index out of range")
        dev_i = lambda a: torch.as_tensor(a, dtype=torch.int32, device=dev)
        self._idx16 = dev_i(self._idx16)
        self._idx32 = dev_i(self._idx32)
        self._buf16 = torch.empty(self._idx16.numel(), dtype=self.dtype, device=dev)
        self._buf32 = torch.empty(self._idx32.numel(), dtype=torch.float32, device=dev)
        self.ctrl_w, self.cbf_w, self.ctrl_rm, self.cbf_rm = [self._buf16[o:o + m] for o, m in v16[:4]]
        self.cbf_rm16, self.cbf_w16, self.ctrl_w16, self.node_rm16 = [self._buf16[o:o + m] for o, m in v16[4:8]]
        self.ctrl_v, self.cbf_v = [self._buf32[o:o + m] for o, m in v32]
        self._cpu_src = None
        self.update()

    @staticmethod
    def _concat(segs, n, align):
        import numpy as np
        out, views, off = [], [], 0
        for a in segs:
            a = np.asarray(a, dtype=np.int64).reshape(-1)
            pad = (-len(a)) % align
            out.append(a)
            out.append(np.full(pad, n, dtype=np.int64))     # padding = constant 0
            views.append((off, len(a)))
            off += len(a) + pad
        return np.concatenate(out), views

    @torch.no_grad()
    def update(self, commit=None):
        """Repack every weight image from the flat parameters. commit (HIP): the deferred commit of
        the optimizer step just enqueued (FlatAdam.step(defer_commit=True)), run in the same launch."""
        if self._buf16.is_cuda:
            from . import native
            native.pack_gather(self.fp.flat, self._idx16, self._buf16, self._idx32, self._buf32, commit=commit)
            return
        n = self.fp.numel
        src = torch.cat([self.fp.flat, torch.tensor([0.0, 1.0], device=self.fp.flat.device)])
        self._buf16.copy_(gather16(src, self._idx16.long(), self.dtype, self.x3))
        self._buf32.copy_(src.index_select(0, self._idx32.long()))
