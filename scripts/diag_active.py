"""Diagnostic: composition of the CBF backward's active evaluation list per iteration.

Counts, after each train_step at the headline config, the deduplicated evaluations (nev), the
active ones (dh != 0) and how many of those are self slots (kNN slot 0: the pair (i, i), whose
input is the same constant for every agent), plus h of a self evaluation.
Usage: python scripts/diag_active.py [--iters 12] [--agents 1024] [--envs 64] [--dtype fp32]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from macbf_gnn_amd import config as C  # noqa: E402
from macbf_gnn_amd.engine import Trainer  # noqa: E402
from macbf_gnn_amd.parallel.dist import DP  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=12)
ap.add_argument("--agents", type=int, default=1024)
ap.add_argument("--envs", type=int, default=64)
ap.add_argument("--dtype", default="fp32")
args = ap.parse_args()
dev = torch.device("cuda:0")
cfg = C.TrainConfig(num_agents=args.agents, num_envs=args.envs, inner_loops=50, device="hip", seed=0,
                    dtype=args.dtype)
tr = Trainer(cfg, device=dev, dp=DP(device=dev))
eng = tr.engine
for it in range(args.iters):
    st = tr.train_step()
    torch.cuda.synchronize()
    T = int(st["T"])
    B, N, K = eng.B, eng.N, eng.K
    E = T * B * N * K
    nev = int(eng.nev_dev.item())
    nact = int(eng.nact_dev.item())
    act = eng.act_list[:nact].long()
    src = eng.src[: 2 * E].long()
    slot = torch.where(act < E, act % K, src[act.clamp(max=2 * E - 1)] % K)
    nself = int((slot == 0).sum().item())
    hself = float(eng.hbuf[0].item())        # main slot 0 of (t=0, b=0, i=0): the self pair
    print(json.dumps({"it": it, "T": T, "E": E, "nev": nev, "nact": nact, "act_frac": round(nact / nev, 4),
                      "self_active": nself, "self_share_of_active": round(nself / max(nact, 1), 4),
                      "h_self": hself, "loss": round(st["loss_total"], 5)}), flush=True)
