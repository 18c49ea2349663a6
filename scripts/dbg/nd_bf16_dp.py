"""Debug: 3-D bf16 node backward intermediates (dL/dpooled, ego) vs the emulating oracle."""
import sys
import torch
sys.path.insert(0, "tests")
from numerics import ctrl_pool_slots
from macbf_gnn_amd import config as C, env as E, oracle as O
from macbf_gnn_amd.models import Controller
from macbf_gnn_amd.ops import graph, native
from macbf_gnn_amd.ops import layout as L
from macbf_gnn_amd.ops.packing import module_pack

DEV = torch.device("cuda")
for dim, nobs, prec in ((3, 0, torch.bfloat16), (3, 0, torch.float32), (2, 0, torch.bfloat16)):
    torch.manual_seed(dim + nobs)
    ctrl = Controller(2 * dim).to(DEV)
    ctrl.mfma_dtype = prec
    with torch.no_grad():
        for p_ in ctrl.parameters():
            p_.copy_(p_.bfloat16().float())
    s, g, obs = E.generate_scenarios(2, 64, dim=dim, num_obstacles=nobs, seed=9)
    gen = torch.Generator().manual_seed(9)
    s[..., dim:] = (torch.rand(2, 64, dim, generator=gen) - 0.5) * 1.2
    s, g = s.to(DEV).float(), g.to(DEV).float()
    B, N, K = 2, 64, C.TOP_K
    idx = O.knn_idx(s, K, s)
    slots = ctrl_pool_slots(ctrl, s, g, idx)
    mp = module_pack("ctrl", ctrl, DEV)
    w, v, rm = mp.pack(tuple(ctrl.parameters()))
    S = graph.node_records(s, None)
    A = torch.empty(B, N, dim, device=DEV)
    pooled = torch.empty(B, N, L.pooled_row(mp.prec), dtype=w.dtype, device=DEV)
    am = torch.empty(B, N, 128, dtype=torch.uint8, device=DEV)
    native.ctrl_fwd(S, g.contiguous(), idx.to(torch.int32).contiguous(), w, mp.off["ew1f"], mp.off["nw1f"], v, A,
                    None, None, None, pooled=pooled, argmax=am, prec=mp.prec)
    wa = torch.randn(B, N, dim, device=DEV)
    Gn = native.to_records(torch.cat([torch.zeros(B, N, dim, device=DEV), wa / C.TIME_STEP], -1))
    nbn, nbe = native.ctrl_bwd_grids(B * N, DEV)
    pn = torch.empty(nbn, native.CTRL_NODE_PARTIAL, device=DEV)
    dP = torch.zeros(B, N, L.pooled_row(mp.prec), dtype=w.dtype, device=DEV)
    ego = torch.zeros(B, N, S.shape[2], device=DEV)
    native.ctrl_node_bwd(pooled, S, g.contiguous(), A, Gn, None, rm, mp.rm_off, v, 0.0, dP, ego, pn, nbn, prec=mp.prec, init=True)
    torch.cuda.synchronize()
    p = {k: v_.detach().clone().requires_grad_(True) for k, v_ in ctrl.params_dict().items()}
    with O.emulate_bf16(prec == torch.bfloat16):
        aref, aux = O.controller_forward(p, s, g, idx, return_aux=True, pool_slots=slots)
        pl = aux["pooled"]
        gp, = torch.autograd.grad((aref * wa).sum(), [pl])
    dPf = dP[..., :128].float()
    if mp.prec == "fp32":
        dPf = dPf + dP[..., 128:256].float()
    e = ((dPf - gp).norm() / gp.norm()).item()
    diff = (dPf - gp).abs()
    print(dim, mp.prec, f"dP err {e:.3e}", "worst agents", diff.sum(-1).flatten().topk(4).indices.tolist(),
          "per-feature err share top", (diff.sum((0, 1)) / diff.sum()).topk(4).values.tolist())
    pa = (dPf - gp).norm(dim=-1).flatten() / gp.norm(dim=-1).flatten().clamp_min(1e-12)
    print("   per-agent rel err: max", pa.max().item(), "median", pa.median().item(), "n>1e-2", int((pa > 1e-2).sum()))
    bad = (pa > 1e-2).nonzero().flatten().tolist()[:8]
    print("   bad agents", bad)
    for ag in bad[:3]:
        b_, i_ = divmod(ag, N)
        print("    agent", ag, "kernel a", A[b_, i_].tolist(), "ref a", aref[b_, i_].tolist(), "wa", wa[b_, i_].tolist())
