"""Debug: 3-D bf16 controller module gradient vs the emulating oracle (test_modules_nd_obstacles[3-0-bf16])."""
import sys
import torch
sys.path.insert(0, "tests")
from numerics import ctrl_pool_slots
from macbf_gnn_amd import config as C, env as E, oracle as O
from macbf_gnn_amd.models import CBF, Controller

DEV = torch.device("cuda")
for dim, nobs in ((3, 0), (3, 2), (2, 2)):
    torch.manual_seed(dim + nobs)
    ctrl, cbf = Controller(2 * dim).to(DEV), CBF(2 * dim).to(DEV)
    ctrl.mfma_dtype = torch.bfloat16
    with torch.no_grad():
        for p_ in ctrl.parameters():
            p_.copy_(p_.bfloat16().float())
    s, g, obs = E.generate_scenarios(2, 64, dim=dim, num_obstacles=nobs, seed=9)
    gen = torch.Generator().manual_seed(9)
    s[..., dim:] = (torch.rand(2, 64, dim, generator=gen) - 0.5) * 1.2
    s, g = s.to(DEV), g.to(DEV)
    obs = obs.to(DEV) if obs is not None else None
    nodes = O.with_obstacles(s, obs)
    idx = O.knn_idx(s, C.TOP_K, nodes)
    sx = s.clone().requires_grad_(True)
    a = ctrl(sx, g, obstacles=obs)
    wa = torch.randn_like(a)
    (a * wa).sum().backward()
    p = {k: v.detach().clone().requires_grad_(True) for k, v in ctrl.params_dict().items()}
    slots = ctrl_pool_slots(ctrl, s, g, idx, obs)
    with O.emulate_bf16():
        aref, aux = O.controller_forward(p, s, g, idx, nodes=nodes, return_aux=True, pool_slots=slots)
        gr = torch.autograd.grad((aref * wa).sum(), list(p.values()))
    k = aux["gains"]
    print(dim, nobs, "a err", ((a - aref).norm() / aref.norm()).item(), "gain range", k.min().item(), k.max().item())
    for (n_, prm), ref in zip(ctrl.named_parameters(), gr):
        print(f"   {n_:32s} err {((prm.grad - ref).norm() / ref.norm().clamp_min(1e-30)).item():.3e} |ref| {ref.norm().item():.3e} |got| {prm.grad.norm().item():.3e}")
