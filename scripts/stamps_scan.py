"""Phase clocks of the kNN / TTC / safety scan (scan_kernel, diagnostics).

Runs warm-up training iterations at the headline config through the Python rollout loop (so the
per-step scans go through native.scan), captures one step's call, re-runs it with a stamps buffer
and prints, per wave (median over the waves that hold agents): the shader-clock cycles of each
phase and the culling counts (superchunks visited, chunks tested / evaluated / with an insertion).

    python scripts/stamps_scan.py [--envs 64] [--step 8] [--dim 2]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = {0: "env staging", 1: "culling boxes", 2: "setup + bound", 3: "candidate loop", 4: "list merge",
          5: "output slots", 6: "counts"}
# chunk path | cell path (steps of the wave's candidate loop, candidates over its lanes, cell rows in
# its agents' search boxes)
COUNTS = {8: "superchunks visited", 9: "chunks tested|cell steps", 10: "chunks eval.|candidates",
          11: "chunks w/ insertion", 12: "eval. for kNN|rows", 13: "evaluated, safety only"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--step", type=int, default=8)
    ap.add_argument("--warm", type=int, default=2)
    ap.add_argument("--dim", type=int, default=2)
    ap.add_argument("--obstacles", type=int, default=0)
    a = ap.parse_args()
    import torch
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.ops import native

    dev = torch.device("cuda", 0)
    cfg = C.TrainConfig(num_agents=1024, num_envs=a.envs, inner_loops=50, device="hip", seed=0, dim=a.dim,
                        num_obstacles=a.obstacles)
    tr = Trainer(cfg, device=dev)
    tr.engine.native_rollout = False
    calls = []
    orig = native.scan

    def spy(*x, **k):
        if k.get("do_knn", True):
            calls.append((x, dict(k)))
        return orig(*x, **k)

    native.scan = spy
    for _ in range(a.warm):
        calls.clear()
        tr.train_step()
    torch.cuda.synchronize()
    native.scan = orig
    x, k = calls[min(a.step, len(calls) - 1)]
    k = dict(k)
    k["sort"] = True                                 # re-sort the captured step's nodes (later steps moved perm)
    B = x[0].shape[0]
    st = torch.zeros(B * 8192, dtype=torch.int64, device=dev)
    orig(*x, **k)
    orig(*x, stamps=st, **k)
    torch.cuda.synchronize()
    st = st.view(-1, 16).double().cpu()
    live = st[:, :7].sum(1) > 0
    st = st[live]
    med = st.median(dim=0).values
    out = {}
    for i, name in PHASES.items():
        out[name] = round(float(med[i]))
        print(f"  {name:22s} median {float(med[i]):9.0f} cyc   max {float(st[:, i].max()):9.0f}")
    for i, name in COUNTS.items():
        out[name] = float(med[i])
        print(f"  {name:22s} median {float(med[i]):9.1f}       max {float(st[:, i].max()):9.0f}")
    print(json.dumps({"waves": int(live.sum()), "total_median_cycles": round(float(st[:, :7].sum(1).median())),
                      "phases": out}))


if __name__ == "__main__":
    main()
