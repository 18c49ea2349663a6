"""Debug: kernel argmax slots vs oracle max-pool for the 3-D module case."""
import torch
from macbf_gnn_amd import config as C, env as E, oracle as O
from macbf_gnn_amd.models import Controller
from macbf_gnn_amd.ops import graph, native
from macbf_gnn_amd.ops import layout as L
from macbf_gnn_amd.ops.packing import module_pack

DEV = torch.device("cuda")
for dim, nobs, N in ((3, 0, 64), (2, 0, 64)):
    torch.manual_seed(dim + nobs)
    ctrl = Controller(2 * dim).to(DEV)
    s, g, obs = E.generate_scenarios(2, N, dim=dim, num_obstacles=nobs, seed=9)
    gen = torch.Generator().manual_seed(9)
    s[..., dim:] = (torch.rand(2, N, dim, generator=gen) - 0.5) * 1.2
    s, g = s.to(DEV).float(), g.to(DEV).float()
    idx = O.knn_idx(s, C.TOP_K, s)
    B, K = 2, C.TOP_K
    mp = module_pack("ctrl", ctrl, DEV)
    w, v, rm = mp.pack(list(ctrl.parameters()))
    S = graph.node_records(s, None)
    A = torch.empty(B, N, dim, device=DEV)
    pooled = torch.empty(B, N, L.pooled_row(mp.prec), dtype=w.dtype, device=DEV)
    am = torch.empty(B, N, 128, dtype=torch.uint8, device=DEV)
    native.ctrl_fwd(S, g.contiguous(), idx.to(torch.int32).contiguous(), w, mp.off["ew1f"], mp.off["nw1f"], v, A,
                    None, None, None, pooled=pooled, argmax=am, prec=mp.prec)
    torch.cuda.synchronize()
    p = {k: v_.detach() for k, v_ in ctrl.params_dict().items()}
    rel, eye = O.edge_rel(s, idx, s)
    x = torch.cat([rel, eye.unsqueeze(-1)], -1)
    dist = torch.sqrt(O.sq_dist(rel, dim))
    mask = (dist < C.OBS_RADIUS).float()
    h = torch.relu(O._lin(x, p["controller_centr_net.0.weight"], p["controller_centr_net.0.bias"], first=True))
    h = torch.relu(O._lin(h, p["controller_centr_net.2.weight"], p["controller_centr_net.2.bias"]))
    hm = h * mask.unsqueeze(-1)                       # (B,N,K,128)
    pv, pi = hm.max(dim=-2)
    amk = am.long()
    has = amk != 255
    print(dim, nobs, "pooled>0:", (pv > 0).float().mean().item(), "kernel has slot:", has.float().mean().item())
    print("  slot present where pooled==0:", (has & (pv == 0)).sum().item(), " missing where pooled>0:", (~has & (pv > 0)).sum().item())
    both = has & (pv > 0)
    diff = both & (amk != pi)
    print("  argmax differs:", diff.sum().item(), "of", both.sum().item())
    if diff.any():
        b, i, c = diff.nonzero()[0].tolist()
        print("   e.g. b,i,c", b, i, c, "kernel slot", amk[b, i, c].item(), "oracle", pi[b, i, c].item(),
              "vals", hm[b, i, :, c].tolist(), "idx", idx[b, i].tolist(), "mask", mask[b, i].tolist())
    # values at slot where pooled==0 but kernel slot present
    bad = has & (pv == 0)
    if bad.any():
        b, i, c = bad.nonzero()[0].tolist()
        sl = amk[b, i, c].item()
        print("   zero-pool slot", sl, "h", h[b, i, sl, c].item(), "mask", mask[b, i, sl].item(), "dist", dist[b, i, sl].item())
