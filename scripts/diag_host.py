"""Host-side (Python + launch) cost of one training iteration (diagnostics, not a benchmark).

Small configurations (config #2: 32 agents x 1 env) are host-bound between the rollout's horizon
read-back and the next rollout launch: this prints the wall time per iteration, then the cProfile
table (tottime) of the same loop, so the Python / launch work on that path can be ranked.

    python scripts/diag_host.py [--agents 32] [--envs 1] [--dtype bf16] [--steps 50] [--top 30]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=32)
    ap.add_argument("--envs", type=int, default=1)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    import torch
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd.engine import Trainer

    dev = torch.device("cuda", 0)
    tr = Trainer(C.TrainConfig(num_agents=a.agents, num_envs=a.envs, device="hip", seed=0, dtype=a.dtype), device=dev)
    for _ in range(a.warmup):
        tr.train_step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.train_step()
    torch.cuda.synchronize()
    print(f"wall {1e3 * (time.perf_counter() - t0) / a.steps:.3f} ms / iteration")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        tr.train_step()
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(a.top)
    print(s.getvalue())
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(a.top)
    print(s.getvalue())


if __name__ == "__main__":
    main()
