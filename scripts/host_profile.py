"""Host-side (Python) cost of the training step: cProfile over a few iterations of the headline
config. The GPU runs ahead of the host except where the host synchronises (early-stop check), so
host time per launch shows up as GPU idle gaps after each synchronisation.

usage: python scripts/host_profile.py [--steps 5] [--top 40]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--top", type=int, default=40)
ap.add_argument("--agents", type=int, default=1024)
ap.add_argument("--envs", type=int, default=64)
args = ap.parse_args()

import torch  # noqa: E402

from macbf_gnn_amd import config as C  # noqa: E402
from macbf_gnn_amd.engine import Trainer  # noqa: E402
from macbf_gnn_amd.parallel import DP  # noqa: E402

dev = torch.device("cuda")
cfg = C.TrainConfig(num_agents=args.agents, num_envs=args.envs, inner_loops=50, device="hip", seed=0)
tr = Trainer(cfg, device=dev, dp=DP(device=dev))
for _ in range(3):
    tr.train_step()
torch.cuda.synchronize()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
for _ in range(args.steps):
    tr.train_step()
pr.disable()
torch.cuda.synchronize()
print(f"wall per step {1e3 * (time.perf_counter() - t0) / args.steps:.3f} ms")
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(args.top)
