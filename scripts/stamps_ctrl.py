"""Phase clocks of the fp32 (x3) controller step, ctrl_fwd_kernel (diagnostics).

Runs warm-up training iterations at the headline config through the Python rollout loop (so the
per-step launches go through native.ctrl_fwd), captures one step's call, re-runs it with a stamps
buffer and prints the shader-clock cycles of each phase: median over waves of the per-wave sums
(the per-tile phases summed over the wave's edge tiles; per tile in the last column).

    python scripts/stamps_ctrl.py [--envs 64] [--step 8]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = {0: "weights", 1: "prologue loads", 2: "tile load issue", 3: "edge features", 4: "edge MLP",
          5: "pool + stores", 6: "pooled-store wait", 7: "node phase"}
PER_TILE = (2, 3, 4, 5)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--step", type=int, default=8)
    ap.add_argument("--warm", type=int, default=2)
    a = ap.parse_args()
    import torch
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.ops import native

    dev = torch.device("cuda", 0)
    tr = Trainer(C.TrainConfig(num_agents=1024, num_envs=a.envs, inner_loops=50, device="hip", seed=0), device=dev)
    tr.engine.native_rollout = False
    calls = []
    orig = native.ctrl_fwd

    def spy(*x, **k):
        calls.append((x, dict(k)))
        return orig(*x, **k)

    native.ctrl_fwd = spy
    for _ in range(a.warm):
        calls.clear()
        tr.train_step()
    torch.cuda.synchronize()
    native.ctrl_fwd = orig
    x, k = calls[min(a.step, len(calls) - 1)]
    st = torch.zeros(2 * native.num_cu(dev) * 8 * 16, dtype=torch.int64, device=dev)
    orig(*x, **k)                                   # warm the caches as in the rollout
    orig(*x, stamps=st, **k)
    torch.cuda.synchronize()
    st = st.view(-1, 16).double().cpu()
    live = st[:, 15] > 0                             # waves that ran a group
    st = st[live]
    tiles = float(st[:, 15].median())
    med = st.median(dim=0).values
    rows = {}
    for i, name in PHASES.items():
        v = float(med[i])
        rows[name] = round(v)
        per = f"   per tile {v / tiles:8.0f}" if i in PER_TILE else ""
        print(f"  {name:18s} median {v:9.0f} cyc   max {float(st[:, i].max()):9.0f}{per}")
    total = float(st[:, :8].sum(1).median())
    print(json.dumps({"waves": int(live.sum()), "tiles_per_wave": tiles, "total_median_cycles": round(total),
                      "phases_median_cycles": rows}))


if __name__ == "__main__":
    main()
