"""CBF forward/backward on the HIP device as a ``torch.autograd.Function``.

Used by ``models.CBF.forward`` on gfx950 (the reference-compatible module API, ``cbf.py:21-45``).
Forward: ``cbf_fwd`` (MFMA edge MLP, radius mask) on the kNN slots. Backward: ``cbf_bwd``
(recompute + hand-written backward, per-WG dW slabs), ``rev_csr`` + ``node_reduce``
(deterministic edge -> node gather for dL/ds), ``reduce_rows`` + the layout's gradient map for
the parameter gradients. No PyTorch autograd inside; no fallback.
"""
from __future__ import annotations

import torch

from .. import config as C
from . import graph, native
from .packing import module_pack


def _edge_mask(s, idx):
    """Radius mask d_eps(i, j) <= OBS_RADIUS of every slot (fp32, as in the kernels)."""
    B, N, K = idx.shape
    sj = s[..., :2].gather(1, idx.long().reshape(B, N * K, 1).expand(B, N * K, 2)).view(B, N, K, 2)
    rel = s[..., :2].unsqueeze(2) - sj
    d = torch.sqrt(rel[..., 0] * rel[..., 0] + rel[..., 1] * rel[..., 1] + C.CBF_DIST_EPS)
    return d <= C.OBS_RADIUS


class _CBFFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, idx, mp, *params):
        B, N, K = idx.shape
        w, v, rm = mp.pack(params)
        S = s.detach().float().contiguous().view(1, B, N, 4)
        idx1 = idx.view(1, B, N, K)
        h = torch.empty(1, B, N, K, dtype=torch.float32, device=s.device)
        native.cbf_fwd(S, idx1, w, mp.off["w1f"], v, two=False, h_out=h)
        ctx.mp = mp
        ctx.packed = (w, v, rm)
        ctx.save_for_backward(S, idx1)
        return h.view(B, N, K)

    @staticmethod
    def backward(ctx, gh):
        S, idx1 = ctx.saved_tensors
        mp = ctx.mp
        w, v, rm = ctx.packed
        _, B, N, K = idx1.shape
        dev = S.device
        dh = (gh.float() * _edge_mask(S[0], idx1[0])).contiguous().view(1, 1, B, N, K)
        dE = torch.empty(1, 1, B, N, K, 4, dtype=torch.float32, device=dev)
        nb = native.cbf_bwd_grid(B * N * K, dev)
        part = torch.empty(nb, native.CBF_PARTIAL, dtype=torch.float32, device=dev)
        native.cbf_bwd(S, idx1, dh, w, mp.off["w1f"], rm, v, passes=1, dE=dE, partial=part, num_blocks=nb)
        gs = None
        if ctx.needs_input_grad[0]:
            rptr = torch.empty(B, N + 1, dtype=torch.int32, device=dev)
            red_e = torch.empty(B, N * K, dtype=torch.int32, device=dev)
            native.rev_csr(idx1.view(B, N, K), rptr, red_e)
            out = torch.zeros(2, B, N, 4, dtype=torch.float32, device=dev)
            native.node_reduce(dE, rptr, red_e, out, T=1, B=B, N=N, K=K, passes=1)
            gs = out[0]
        red = torch.empty(native.CBF_PARTIAL, dtype=torch.float32, device=dev)
        native.reduce_rows(part, red)
        pgrads = mp.unpack_grads({"cbf": red})
        return (gs, None, None, *pgrads)


def cbf_apply(module, s: torch.Tensor, idx: torch.Tensor | None, top_k: int = C.TOP_K) -> torch.Tensor:
    """s (B, N, 4) on the HIP device -> h (B, N, K) (radius-masked), differentiable in s and
    in the module's parameters."""
    lead = s.shape[:-2]
    N = s.shape[-2]
    s3 = s.reshape(-1, N, 4)
    if idx is None:
        idx3 = graph.knn(s3, top_k)
    else:
        idx3 = idx.reshape(-1, N, idx.shape[-1]).to(torch.int32).contiguous()
    mp = module_pack("cbf", module, s.device)
    h = _CBFFn.apply(s3.float(), idx3, mp, *module.parameters())
    return h.reshape(*lead, N, idx3.shape[-1])
