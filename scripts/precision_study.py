"""How well-conditioned are the training-step gradients? (why do the 4,096-agent and
3-D + obstacle fp32 comparisons sit at ~4e-4 while most sit near 1e-5?)

Runs the pure-torch oracle step (autograd through the rollout, CPU) in fp32 and again in fp64 on
the fp32 run's trajectory (same states, neighbour graphs), and reports per parameter tensor the
relative norm difference |g32 - g64| / |g64| -- the error of an exact-fp32 implementation of the
step itself -- next to the cancellation ratio sum|per-edge terms| / |sum| is not needed: a
large fp32-vs-fp64 gap is the conditioning.

    python scripts/precision_study.py --agents 4096 --envs 2 --steps 3
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def grads(tr, s0, g, dtype, forced=None):
    import torch
    from macbf_gnn_amd import oracle
    cfg = tr.cfg
    cp = {k: v.detach().to(dtype).requires_grad_(True) for k, v in tr.controller.params_dict().items()}
    bp = {k: v.detach().to(dtype).requires_grad_(True) for k, v in tr.cbf.params_dict().items()}
    s0, g = s0.to(dtype), g.to(dtype)
    traj = oracle.rollout(cp, s0, g, top_k=cfg.top_k, inner_loops=cfg.inner_loops, bptt=cfg.bptt,
                          early_stop=cfg.early_stop, compute_safety=False, forced=forced)
    T = traj["A"].shape[1]
    valid = traj["valid"]
    s_d = traj["S"][:, :T].detach()
    dang = oracle.ttc_mask_knn(s_d, traj["idx"])
    vmask = valid[..., None, None]
    N = s0.shape[1]
    n = {"n_dang": float((dang & vmask).sum()), "n_safe": float((~dang & vmask).sum()),
         "n_act": float(valid.sum() * N)}
    losses, _, _ = oracle.train_losses(cp, bp, traj, g, n_counts=n, reuse_nbr_idx=cfg.reuse_nbr_idx, top_k=cfg.top_k)
    names = list(cp) + list(bp)
    gr = torch.autograd.grad(losses["total"], [*cp.values(), *bp.values()])
    return dict(zip(names, gr)), traj


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=4096)
    ap.add_argument("--envs", type=int, default=2)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    import torch
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd.engine import Trainer
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    cfg = C.TrainConfig(num_agents=a.agents, num_envs=a.envs, inner_loops=a.steps, early_stop=False, seed=a.seed,
                        device="cpu")
    tr = Trainer(cfg)
    s0, g, _ = tr.sample()
    g32, traj = grads(tr, s0, g, torch.float32)
    forced = {"S": traj["S"].detach().double(), "idx": traj["idx"]}
    g64, _ = grads(tr, s0, g, torch.float64, forced=forced)
    rel = {k: float((g32[k].double() - g64[k]).norm() / g64[k].norm().clamp_min(1e-300)) for k in g64}
    worst = sorted(rel.items(), key=lambda kv: -kv[1])
    print(json.dumps({"agents": a.agents, "envs": a.envs, "steps": a.steps,
                      "worst": [(k, f"{v:.2e}") for k, v in worst[:5]],
                      "median": f"{sorted(rel.values())[len(rel) // 2]:.2e}"}))


if __name__ == "__main__":
    main()
