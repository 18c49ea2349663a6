"""GNN controller forward/backward on the HIP device as a ``torch.autograd.Function``.

Used by ``models.Controller.forward`` on gfx950 (reference ``controller.py:31-63``).
Forward: ``ctrl_fwd`` (edge MLP + masked max-pool with saved argmax slots + node MLP + gain
law), no Euler step. Backward: ``ctrl_node_bwd`` (node MLP + gain law; the upstream dL/da is
fed as the velocity adjoint of s_{t+1} = s_t + dt [v, a], i.e. G = (0, 0, dL/da / dt)),
``ctrl_edge_bwd`` (max-pool routing via argmax, edge MLP), ``node_combine`` (edge -> node,
reverse CSR, no Euler term) and the slab reductions for the parameter gradients.

Goals enter only through p - g (node-MLP input and the PD law), so dL/dg is minus the position
part of the node-path adjoint ``ego`` (reference: autograd through ``controller.py:47,54-61``).
Precision: the module's ``mfma_dtype`` (default torch.float32 = the fp32-accurate x3 kernels).
"""
from __future__ import annotations

import torch

from .. import config as C
from . import graph, native
from . import layout as L
from .packing import module_pack


class _CtrlFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, g, obs, idx, mp, *params):
        B, N, K = idx.shape
        D = mp.dim
        dev = s.device
        w, v, rm = mp.pack(params)
        S = graph.node_records(s, obs)                   # (B, Nn, W)
        G = g.detach().float().contiguous()
        A = torch.empty(B, N, D, dtype=torch.float32, device=dev)
        pooled = torch.empty(B, N, L.pooled_row(mp.prec), dtype=w.dtype, device=dev)
        am = torch.empty(B, N, 128, dtype=torch.uint8, device=dev)
        native.ctrl_fwd(S, G, idx, w, mp.off["ew1f"], mp.off["nw1f"], v, A, None, None, None,
                        pooled=pooled, argmax=am, prec=mp.prec)
        ctx.mp = mp
        ctx.packed = (w, v, rm)
        ctx.save_for_backward(S, G, idx, A, pooled, am)
        return A

    @staticmethod
    def backward(ctx, gA):
        S, G, idx, A, pooled, am = ctx.saved_tensors
        mp = ctx.mp
        w, v, rm = ctx.packed
        B, N, K = idx.shape
        Nn, W = S.shape[1], S.shape[2]
        D = mp.dim
        dev = S.device
        Gn = native.to_records(torch.cat([torch.zeros(B, N, D, device=dev), gA.float() / C.TIME_STEP], -1))
        nbn, nbe = native.ctrl_bwd_grids(B * N, dev, mp.prec)
        # one step: the kernels write their slabs (init) instead of accumulating
        pn = torch.empty(nbn, native.CTRL_NODE_PARTIAL, dtype=torch.float32, device=dev)
        pe = torch.empty(nbe, native.CTRL_EDGE_PARTIAL, dtype=torch.float32, device=dev)
        dP = torch.empty(B, N, L.pooled_row(mp.prec), dtype=w.dtype, device=dev)
        ego = torch.empty(B, N, W, dtype=torch.float32, device=dev)
        dEc = torch.empty(B, N, K, W, dtype=torch.float32, device=dev)
        native.ctrl_node_bwd(pooled, S, G, A, Gn, None, rm, mp.rm_off, v, 0.0, dP, ego, pn, nbn, prec=mp.prec, init=True)
        native.ctrl_edge_bwd(S, idx, am, dP, w, mp.off["ew1f"], mp.off["ew2tn"], dEc, pe, nbe, prec=mp.prec, init=True)
        gs = gg = None
        if ctx.needs_input_grad[1]:
            # goals only enter through p - g: dL/dg = -dL/d(p - g) of the node path
            gg = -native.from_records(ego)[..., :D]
        if ctx.needs_input_grad[0]:
            rptr = torch.empty(B, Nn + 1, dtype=torch.int32, device=dev)
            red_e = torch.empty(B, N * K, dtype=torch.int32, device=dev)
            native.rev_csr(idx, rptr, red_e, n_nodes=Nn)
            gsr = torch.empty(B, N, W, dtype=torch.float32, device=dev)
            native.node_combine(torch.zeros(B, N, W, device=dev), ego, dEc, rptr, red_e, None, gsr, K=K)
            gs = native.from_records(gsr)
        rn = torch.empty(native.CTRL_NODE_PARTIAL, dtype=torch.float32, device=dev)
        re = torch.empty(native.CTRL_EDGE_PARTIAL, dtype=torch.float32, device=dev)
        native.reduce_rows(pn, rn)
        native.reduce_rows(pe, re)
        pgrads = mp.unpack_grads({"node": rn, "edge": re})
        return (gs, gg, None, None, None, *pgrads)


def controller_apply(module, s: torch.Tensor, g: torch.Tensor, idx: torch.Tensor | None,
                     top_k: int = C.TOP_K, obstacles: torch.Tensor | None = None) -> torch.Tensor:
    """s (..., N, 2D), g (..., N, D) on the HIP device -> a (..., N, D); differentiable in s, g and
    the module's parameters (obstacles are constants)."""
    lead = s.shape[:-2]
    N, SD = s.shape[-2:]
    D = SD // 2
    s3 = s.reshape(-1, N, SD)
    g3 = g.reshape(-1, N, D)
    obs = None
    if obstacles is not None:
        obs = obstacles if obstacles.dim() == 3 else obstacles.unsqueeze(0)
        obs = obs.expand(s3.shape[0], *obs.shape[-2:]).float()
    if idx is None:
        idx3 = graph.knn(s3, top_k, obs)
    else:
        idx3 = idx.reshape(-1, N, idx.shape[-1]).to(torch.int32).contiguous()
    mp = module_pack("ctrl", module, s.device)
    a = _CtrlFn.apply(s3.float(), g3.float(), obs, idx3, mp, *module.parameters())
    return a.reshape(*lead, N, D)
