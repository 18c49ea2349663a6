"""Config #2 (32 agents x 1 env) iteration time vs the edge backward's tile split and the per-step
slab rows of small BPTT grids (diagnostics).

native.ctrl_edge_qsplit picks how many workgroups share a small scene's edge-backward tile rounds
(16 at 32 agents: 12 tiles, 4 workgroups idle but each writes its zero slab row). Every variant
gets its own trainer (the split is fixed when the engine is built); one process, interleaved reps.

    python scripts/diag_qsplit.py [--dtype bf16] [--splits 16/12/8 (or commas)] [--step_rows 1/0] [--reps 2]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--agents", type=int, default=32)
    ap.add_argument("--envs", type=int, default=1)
    ap.add_argument("--splits", default="16,12,8,6,4")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--step_rows", default="1")
    a = ap.parse_args()
    import torch
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.ops import native
    from macbf_gnn_amd.engine import hip_engine

    dev = torch.device("cuda", 0)
    orig = native.ctrl_edge_qsplit
    out = {}
    for rep in range(a.reps):
        for q, sr in [(int(x), int(y)) for x in a.splits.replace("/", ",").split(",") for y in a.step_rows.replace("/", ",").split(",")]:
            native.ctrl_edge_qsplit = lambda total, device, q=q: q
            hip_engine.STEP_ROWS_BYTES = (64 << 20) if sr else 0
            tr = Trainer(C.TrainConfig(num_agents=a.agents, num_envs=a.envs, device="hip", seed=0, dtype=a.dtype),
                         device=dev)
            for _ in range(a.warmup):
                tr.train_step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                tr.train_step()
            torch.cuda.synchronize()
            out[f"q{q}_sr{sr}_{rep}"] = round((time.perf_counter() - t0) / a.steps * 1e3, 4)
            del tr
    native.ctrl_edge_qsplit = orig
    print(json.dumps(out))


if __name__ == "__main__":
    main()
