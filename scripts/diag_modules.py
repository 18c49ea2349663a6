"""Per-parameter relative gradient errors of the native module path vs the fp32 oracle."""
import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from macbf_gnn_amd import config as C, env as E, oracle as O
from macbf_gnn_amd.models import CBF, Controller
DEV = torch.device("cuda")


def rel(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


for dim, B, N in ((2, 2, 64), (3, 2, 64), (2, 4, 512), (3, 4, 512)):
    torch.manual_seed(0)
    ctrl = Controller(2 * dim).to(DEV)
    with torch.no_grad():
        for p in ctrl.parameters():
            p.copy_(p.bfloat16().float())
    s, g, _ = E.generate_scenarios(B, N, dim=dim, seed=9)
    gen = torch.Generator().manual_seed(1)
    s[..., dim:] = (torch.rand(B, N, dim, generator=gen) - 0.5) * 1.2
    s, g = s.to(DEV), g.to(DEV)
    idx = O.knn_idx(s, 12)
    sx = s.clone().requires_grad_(True)
    a = ctrl(sx, g)
    w = torch.randn_like(a)
    (a * w).sum().backward()
    p = {k: v.detach().clone().requires_grad_(True) for k, v in ctrl.params_dict().items()}
    s2 = s.clone().requires_grad_(True)
    aref = O.controller_forward(p, s2, g, idx)
    gr = torch.autograd.grad((aref * w).sum(), [s2] + list(p.values()))
    errs = {"a": rel(a.detach(), aref.detach()), "ds": rel(sx.grad, gr[0])}
    for (k, prm), ref in zip(ctrl.named_parameters(), gr[1:]):
        errs[k.replace("controller_", "")] = rel(prm.grad, ref)
    print(dim, B, N, " ".join(f"{k}={v:.3f}" for k, v in errs.items()), flush=True)
