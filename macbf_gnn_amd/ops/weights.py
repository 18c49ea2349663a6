"""Per-step repacking of the flat fp32 master parameters into the kernels' bf16 MFMA
fragment buffers (+ fp32 side vectors). One gather per network per optimizer step."""
from __future__ import annotations

import torch

from . import layout as L


class PackedWeights:
    def __init__(self, fp, dim: int = 2, dtype=torch.bfloat16):
        self.fp = fp
        self.dim = dim
        self.dtype = dtype
        offs = {pn: o for (m, pn, shape, o, n) in fp.specs}
        dev = fp.flat.device
        n = fp.numel
        self.ctrl_pk = L.ctrl_packer(offs, dim)
        self.cbf_pk = L.cbf_packer(offs, dim)
        self.ctrl_off = self.ctrl_pk.offsets()
        self.cbf_off = self.cbf_pk.offsets()
        cv, self.ctrl_voff = L.ctrl_vec_index(offs, dim)
        bv, self.cbf_voff = L.cbf_vec_index(offs)
        mk = lambda a: torch.as_tensor(L.resolve(a, n), dtype=torch.long, device=dev)
        self._ictrl = mk(self.ctrl_pk.index())
        self._icbf = mk(self.cbf_pk.index())
        self._vctrl = mk(cv)
        self._vcbf = mk(bv)
        self.node_rm = L.ctrl_node_rm(offs, dim)
        self.node_rm_off = self.node_rm.offsets()
        self._irm = mk(self.node_rm.index())
        self.cbf_rmp = L.cbf_rm(offs)
        self._icrm = mk(self.cbf_rmp.index())
        self._src = torch.zeros(n + 2, dtype=torch.float32, device=dev)
        self._src[n + 1] = 1.0
        self.ctrl_w = torch.empty(self._ictrl.numel(), dtype=dtype, device=dev)
        self.cbf_w = torch.empty(self._icbf.numel(), dtype=dtype, device=dev)
        self.ctrl_v = torch.empty(self._vctrl.numel(), dtype=torch.float32, device=dev)
        self.cbf_v = torch.empty(self._vcbf.numel(), dtype=torch.float32, device=dev)
        self.ctrl_rm = torch.empty(self._irm.numel(), dtype=dtype, device=dev)
        self.cbf_rm = torch.empty(self._icrm.numel(), dtype=dtype, device=dev)
        self.update()

    @torch.no_grad()
    def update(self):
        n = self.fp.numel
        self._src[:n].copy_(self.fp.flat)
        self.ctrl_w.copy_(self._src.index_select(0, self._ictrl))
        self.cbf_w.copy_(self._src.index_select(0, self._icbf))
        torch.index_select(self._src, 0, self._vctrl, out=self.ctrl_v)
        torch.index_select(self._src, 0, self._vcbf, out=self.cbf_v)
        self.ctrl_rm.copy_(self._src.index_select(0, self._irm))
        self.cbf_rm.copy_(self._src.index_select(0, self._icrm))
