"""Critical-path cost of the side-stream scenario sampler (diagnostics, not a benchmark).

Times the headline training iteration twice on one trainer: as bench.py runs it (the next
iteration's scenarios sampled on a side stream), then with the sampler removed from the loop
(every iteration reuses one pre-sampled scenario set -- NOT a valid benchmark, the workload's data
stops changing). The difference bounds what a faster or differently placed sampler could save.

    python scripts/diag_sampler.py [--envs 64] [--steps 20] [--warmup 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import torch
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd.engine import Trainer

    dev = torch.device("cuda", 0)
    tr = Trainer(C.TrainConfig(num_agents=1024, num_envs=a.envs, device="hip", seed=0), device=dev)

    def window():
        for _ in range(a.warmup):
            tr.train_step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            tr.train_step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps * 1e3

    out = {"envs": a.envs}
    orig = tr._take_sample
    fixed = tr.sample()
    torch.cuda.synchronize()
    for rep in range(a.reps):
        tr._take_sample = orig
        out[f"sampler_{rep}"] = round(window(), 3)
        tr._take_sample = lambda: fixed
        out[f"no_sampler_{rep}"] = round(window(), 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
