"""Fixed, deterministic training workload for the profiler checks (SURVEY 4.6,
tests/test_gpu_profiler.py): the fp32 (x3) HIP engine at 512 agents x 8 envs, fixed horizon (no
early stop: every run issues the same launches), seed 0, ``--iters`` full training iterations
after one warm-up iteration. Run it under ``rocprofv3`` with this program right after ``--``.

    python scripts/prof_workload.py [--iters 2] [--dtype fp32] [--agents 512 --envs 8]

With ``--summarize PMC_CSV [PMC_CSV ...] --out JSON`` it instead folds rocprofv3 ``--pmc`` CSV
outputs into per-kernel per-dispatch averages (the baseline format of the test).
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIG = dict(num_agents=512, num_envs=8, inner_loops=6, seed=0, early_stop=False)


def kernel_key(name: str) -> str:
    """'void mb::x3::ctrl_fwd_kernel<8, 2, true>(mb::CtrlArgs)' -> 'mb::x3::ctrl_fwd_kernel<8, 2, true>'"""
    n = name.split("(")[0]
    return n[5:] if n.startswith("void ") else n


def summarize(paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.defaultdict(int))
    for p in paths:
        for x in csv.DictReader(open(p)):
            k = kernel_key(x["Kernel_Name"])
            agg[k][x["Counter_Name"]] += float(x["Counter_Value"])
            cnt[k][x["Counter_Name"]] += 1
    return {k: {c: v / cnt[k][c] for c, v in row.items()} | {"dispatches": max(cnt[k].values())}
            for k, row in agg.items()}


def run(iters, dtype, agents=None, envs=None):
    # no start-up self-check: its kernel launches would enter the per-dispatch counter averages
    os.environ.setdefault("MACBF_SELFCHECK", "0")
    import torch
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd.engine import Trainer
    conf = dict(CONFIG)
    if agents:
        conf["num_agents"] = agents
    if envs:
        conf["num_envs"] = envs
    cfg = C.TrainConfig(device="hip", dtype=dtype, display_steps=10 ** 9, save_steps=10 ** 9, **conf)
    tr = Trainer(cfg)
    for _ in range(iters + 1):
        tr.train_step()
    torch.cuda.synchronize()
    print(json.dumps({"iters": iters, "dtype": dtype, **conf}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--agents", type=int, default=None)
    ap.add_argument("--envs", type=int, default=None)
    ap.add_argument("--summarize", nargs="*", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.summarize is not None:
        s = summarize(a.summarize)
        if a.out:
            json.dump(s, open(a.out, "w"), indent=1, sort_keys=True)
        print(json.dumps(s, indent=1, sort_keys=True))
        return
    run(a.iters, a.dtype, a.agents, a.envs)


if __name__ == "__main__":
    main()
