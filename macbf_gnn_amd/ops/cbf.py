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
from .. import oracle
from . import graph, native
from .packing import module_pack


def _edge_mask(S, idx, D):
    """Radius mask d_eps(i, j) <= OBS_RADIUS of every slot (fp32, as in the kernels); S are the
    (B, Nn, W) node records (positions in the first D columns)."""
    B, N, K = idx.shape
    P = S[..., :D]
    pj = P.gather(1, idx.long().reshape(B, N * K, 1).expand(B, N * K, D)).view(B, N, K, D)
    rel = P[:, :N].unsqueeze(2) - pj
    d = torch.sqrt(oracle.sq_dist(rel, D) + C.CBF_DIST_EPS_COORD * D)
    return d <= C.OBS_RADIUS


class _CBFFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, obs, idx, mp, *params):
        B, N, K = idx.shape
        w, v, rm = mp.pack(params)
        Sr = graph.node_records(s, obs)                  # (B, Nn, W)
        S = Sr.view(1, *Sr.shape)
        idx1 = idx.view(1, B, N, K)
        h = torch.empty(1, B, N, K, dtype=torch.float32, device=s.device)
        native.cbf_fwd(S, idx1, w, mp.off["w1f"], v, two=False, h_out=h, prec=mp.prec)
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
        Nn, W = S.shape[2], S.shape[3]
        D = mp.dim
        dev = S.device
        dh = (gh.float() * _edge_mask(S[0], idx1[0], D)).contiguous().view(1, 1, B, N, K)
        dE = torch.empty(1, 1, B, N, K, W, dtype=torch.float32, device=dev)
        nb = native.cbf_bwd_grid(B * N * K, dev)
        part = torch.empty(nb, native.CBF_PARTIAL, dtype=torch.float32, device=dev)
        native.cbf_bwd(S, idx1, dh, w, mp.off["w1f"], rm, v, passes=1, dE=dE, partial=part, num_blocks=nb,
                       prec=mp.prec)
        gs = None
        if ctx.needs_input_grad[0]:
            rptr = torch.empty(B, Nn + 1, dtype=torch.int32, device=dev)
            red_e = torch.empty(B, N * K, dtype=torch.int32, device=dev)
            native.rev_csr(idx1.view(B, N, K), rptr, red_e, n_nodes=Nn)
            out = torch.zeros(2, B, N, W, dtype=torch.float32, device=dev)
            native.node_reduce(dE, rptr, red_e, out, T=1, B=B, N=N, K=K, passes=1, n_nodes=Nn)
            gs = native.from_records(out[0])
        red = torch.empty(native.CBF_PARTIAL, dtype=torch.float32, device=dev)
        native.reduce_rows(part, red)
        pgrads = mp.unpack_grads({"cbf": red})
        return (gs, None, None, None, *pgrads)


def cbf_apply(module, s: torch.Tensor, idx: torch.Tensor | None, top_k: int = C.TOP_K,
              obstacles: torch.Tensor | None = None) -> torch.Tensor:
    """s (..., N, 2D) on the HIP device -> h (..., N, K) (radius-masked), differentiable in s and
    in the module's parameters; obstacles (B, M, D) join the graph as static nodes."""
    lead = s.shape[:-2]
    N, SD = s.shape[-2:]
    s3 = s.reshape(-1, N, SD)
    obs = None
    if obstacles is not None:
        obs = obstacles if obstacles.dim() == 3 else obstacles.unsqueeze(0)
        obs = obs.expand(s3.shape[0], *obs.shape[-2:]).float()
    if idx is None:
        idx3 = graph.knn(s3, top_k, obs)
    else:
        idx3 = idx.reshape(-1, N, idx.shape[-1]).to(torch.int32).contiguous()
    mp = module_pack("cbf", module, s.device)
    h = _CBFFn.apply(s3.float(), obs, idx3, mp, *module.parameters())
    return h.reshape(*lead, N, idx3.shape[-1])
