"""Debug: 3-D module-API controller gradient (tests/test_gpu_nd.py::test_modules_nd_obstacles[3-0])."""
import torch
from macbf_gnn_amd import config as C, env as E, oracle as O
from macbf_gnn_amd.models import Controller
from macbf_gnn_amd.ops import graph

DEV = torch.device("cuda")
for dim, nobs, N in ((3, 0, 64), (3, 2, 64), (2, 0, 64), (3, 0, 128)):
    torch.manual_seed(dim + nobs)
    ctrl = Controller(2 * dim).to(DEV)
    s, g, obs = E.generate_scenarios(2, N, dim=dim, num_obstacles=nobs, seed=9)
    gen = torch.Generator().manual_seed(9)
    s[..., dim:] = (torch.rand(2, N, dim, generator=gen) - 0.5) * 1.2
    s, g = s.to(DEV), g.to(DEV)
    obs = obs.to(DEV) if obs is not None else None
    nodes = O.with_obstacles(s, obs)
    idx = O.knn_idx(s, C.TOP_K, nodes)
    obs3 = None if obs is None else obs.float()
    idx_k = graph.knn(s, C.TOP_K, obs3).long()
    print(dim, nobs, N, "knn equal:", torch.equal(idx, idx_k))
    sx = s.clone().requires_grad_(True)
    a = ctrl(sx, g, obstacles=obs)
    wa = torch.randn_like(a)
    (a * wa).sum().backward()
    p = {k: v.detach().clone().requires_grad_(True) for k, v in ctrl.params_dict().items()}
    s2 = s.clone().requires_grad_(True)
    aref, aux = O.controller_forward(p, s2, g, idx, nodes=O.with_obstacles(s2, obs), return_aux=True)
    gr = torch.autograd.grad((aref * wa).sum(), [s2] + list(p.values()))
    pooled = aux["pooled"]
    print("  pooled==0 share:", (pooled == 0).float().mean().item(), " mask share:", aux["mask"].mean().item())
    for (k, prm), ref in zip(ctrl.named_parameters(), gr[1:]):
        e = ((prm.grad - ref).norm() / ref.norm()).item()
        if e > 1e-4:
            print(f"  {k}: {e:.3e}  |ref| {ref.norm().item():.3e} |got| {prm.grad.norm().item():.3e} |diff| {(prm.grad-ref).norm().item():.3e}")
            if prm.grad.dim() == 2:
                d = (prm.grad - ref).abs()
                print("    diff col sums:", [round(x, 4) for x in d.sum(0)[:16].tolist()])
                print("    diff row max :", [round(x, 4) for x in d.max(1).values[:16].tolist()])
