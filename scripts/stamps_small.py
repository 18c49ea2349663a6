"""Phase clocks of the persistent small-scene rollout (csrc/ctrl.hip rollout_small_kernel;
diagnostics). Needs a diagnostics build of the controller kernels, e.g.
scripts/build_variant.sh stamps ctrl,ctrl_x3 "-DMB_DIAG=1" and MACBF_EXT=alt_so/stamps/_C.so.
Prints per phase the median over waves of the cycles summed over the rollout's steps and per step.

    python scripts/stamps_small.py [--agents 32] [--envs 1] [--dtype bf16]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = {0: "scan", 1: "edge phase", 2: "barrier", 3: "node phase", 4: "step tail"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=32)
    ap.add_argument("--envs", type=int, default=1)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--warm", type=int, default=3)
    a = ap.parse_args()
    import torch
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd.engine import Trainer

    dev = torch.device("cuda", 0)
    tr = Trainer(C.TrainConfig(num_agents=a.agents, num_envs=a.envs, device="hip", seed=0, dtype=a.dtype), device=dev)
    eng = tr.engine
    assert eng.small_rollout, "not a small-scene config"
    for _ in range(a.warm):
        tr.train_step()
    eng.small_stamps = torch.zeros(a.envs, 8, 16, dtype=torch.int64, device=dev)
    eng._drv = None                       # rebuilt with the stamps buffer
    tr.train_step()
    torch.cuda.synchronize()
    st = eng.small_stamps.view(-1, 16).double().cpu()
    st = st[st[:, 15] > 0]
    steps = float(st[:, 15].median())
    med = st.median(dim=0).values
    out = {"waves": int(st.shape[0]), "steps": steps}
    for k, name in PHASES.items():
        out[name] = round(float(med[k]))
        print(f"  {name:12s} median {float(med[k]):9.0f} cyc   per step {float(med[k]) / max(steps, 1):7.0f}")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
