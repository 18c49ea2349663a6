"""Training-parity run: the HIP engine vs autograd through the fp32 oracle (OracleEngine) on the
same device, same initial weights, same scenarios, for many iterations.

Both trainers start from one seed (identical parameters) and sample the same counter-based
scenarios each iteration; each applies its own gradient to its own parameters, so they follow
their own trajectories. Per iteration the script logs loss terms, accuracies, safety rate and
horizon of both to JSONL, and prints a summary of the last `--window` iterations: mean loss,
accuracies, safety, T and the relative parameter distance between the two runs.

usage: python scripts/parity_run.py --iters 200 --agents 32 --envs 8 --dtype fp32 --out FILE
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=200)
ap.add_argument("--agents", type=int, default=32)
ap.add_argument("--envs", type=int, default=8)
ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
ap.add_argument("--seed", type=int, default=0)
ap.add_argument("--window", type=int, default=50)
ap.add_argument("--out", default="gpurun_out/parity/log.jsonl")
args = ap.parse_args()

import torch  # noqa: E402

from macbf_gnn_amd import config as C  # noqa: E402
from macbf_gnn_amd.engine import Trainer  # noqa: E402
from macbf_gnn_amd.engine.oracle_engine import OracleEngine  # noqa: E402
from macbf_gnn_amd.parallel import DP  # noqa: E402

dev = torch.device("cuda")


def make(oracle):
    cfg = C.TrainConfig(num_agents=args.agents, num_envs=args.envs, inner_loops=C.INNER_LOOPS, device="hip",
                        seed=args.seed, dtype=args.dtype, prefetch_data=False)
    tr = Trainer(cfg, device=dev, dp=DP(device=dev))
    if oracle:
        tr.engine = OracleEngine(tr)
    return tr


hip, orc = make(False), make(True)
assert torch.equal(hip.fp.flat, orc.fp.flat)
KEYS = ["loss_total", "loss_dang", "loss_safe", "loss_dang_deriv", "loss_safe_deriv", "loss_action", "T"]
os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
rows = []
t0 = time.time()
with open(args.out, "w") as f:
    for it in range(args.iters):
        rec = {"iter": it}
        for name, tr in (("hip", hip), ("oracle", orc)):
            st = tr.train_step()
            d = {k: float(st[k]) for k in KEYS}
            nd, ns = max(float(st["n_dang"]), 1.0), max(float(st["n_safe"]), 1.0)
            d["acc_dang"] = float(st["acc_dang_sum"]) / nd
            d["acc_safe"] = float(st["acc_safe_sum"]) / ns
            d["safety"] = float(st["safe_agents"]) / max(float(st["agent_steps"]), 1.0)
            rec[name] = d
        a, b = hip.fp.flat.double(), orc.fp.flat.double()
        rec["param_rel_dist"] = float((a - b).norm() / b.norm())
        rows.append(rec)
        f.write(json.dumps(rec) + "\n")
        if it % 20 == 0:
            print(f"it {it}: hip loss {rec['hip']['loss_total']:.4f} T {rec['hip']['T']:.0f} | oracle loss "
                  f"{rec['oracle']['loss_total']:.4f} T {rec['oracle']['T']:.0f} | param dist {rec['param_rel_dist']:.2e} "
                  f"({time.time() - t0:.0f} s)", flush=True)
w = rows[-args.window:]
summ = {"iters": args.iters, "agents": args.agents, "envs": args.envs, "dtype": args.dtype, "window": len(w)}
for k in KEYS + ["acc_dang", "acc_safe", "safety"]:
    mh = sum(r["hip"][k] for r in w) / len(w)
    mo = sum(r["oracle"][k] for r in w) / len(w)
    summ[k] = {"hip": mh, "oracle": mo, "rel_diff": abs(mh - mo) / max(abs(mo), 1e-12)}
first = rows[: args.window]
summ["loss_total_first_window"] = {"hip": sum(r["hip"]["loss_total"] for r in first) / len(first),
                                   "oracle": sum(r["oracle"]["loss_total"] for r in first) / len(first)}
summ["param_rel_dist_final"] = rows[-1]["param_rel_dist"]
summ["identical_iters_loss_1e-4"] = sum(1 for r in rows if abs(r["hip"]["loss_total"] - r["oracle"]["loss_total"])
                                        <= 1e-4 * abs(r["oracle"]["loss_total"]))
print(json.dumps(summ))
