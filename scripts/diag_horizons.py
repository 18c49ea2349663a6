"""Per-env horizons of the headline training (GPU): for each iteration, T (the max over envs) and
the per-env valid step counts T_b (done masks, reference train.py:78-81 per env), and the share of
the (step, env) grid that is valid -- the work a done-env skip could save in the rollout, the h
forward and the BPTT. usage: python scripts/diag_horizons.py [--iters 25] [--agents 1024 --envs 64]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=25)
    ap.add_argument("--agents", type=int, default=1024)
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--dtype", default="fp32")
    a = ap.parse_args()
    import torch
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd.engine import Trainer
    cfg = C.TrainConfig(num_agents=a.agents, num_envs=a.envs, device="hip", seed=0, dtype=a.dtype)
    tr = Trainer(cfg)
    tot_valid = tot_grid = 0
    for it in range(a.iters):
        st = tr.train_step()
        T = int(float(st["T"]))
        v = tr.engine.valid_buf[:T].to(torch.int64).cpu()
        Tb = v.sum(0).tolist()
        active = [int((v[t] != 0).sum()) for t in range(T)]
        tot_valid += sum(Tb)
        tot_grid += T * a.envs
        print(json.dumps({"it": it, "T": T, "Tb_min": min(Tb), "Tb_mean": sum(Tb) / len(Tb), "valid_share": sum(Tb) / (T * a.envs),
                          "active_envs_per_step": active}), flush=True)
    print(json.dumps({"valid_share_all": tot_valid / tot_grid}))


if __name__ == "__main__":
    main()
