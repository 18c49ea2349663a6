"""Full-step gradient of the fp32 HIP engine vs autograd through the fp32 oracle engine, per
parameter tensor, over seeds / shapes / kernel switches (diagnostics for tests/test_gpu_fp32.py).

    python scripts/diag_fullstep.py --N 12 --B 3 --seeds 0 1 2 --env MACBF_EB16=0
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, nargs="+", default=[12])
    ap.add_argument("--B", type=int, default=3)
    ap.add_argument("--T", type=int, default=5)
    ap.add_argument("--seeds", type=int, nargs="+", default=[0])
    ap.add_argument("--env", nargs="*", default=[])
    a = ap.parse_args()
    for kv in a.env:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    import torch
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.engine.oracle_engine import OracleEngine
    from macbf_gnn_amd.parallel import DP
    dev = torch.device("cuda", 0)
    for N in a.N:
        for seed in a.seeds:
            cfg = C.TrainConfig(num_agents=N, num_envs=a.B, inner_loops=a.T, early_stop=False, seed=seed,
                                device="hip", dtype="fp32")
            tr = Trainer(cfg, device=dev, dp=DP(device=dev))
            s0, g, obs = tr.sample()
            tr.engine.step(s0, g, obs)
            gh = tr.fp.grad.clone().double()
            OracleEngine(tr).step(s0, g, obs)
            go = tr.fp.grad.clone().double()
            errs = {}
            for m, pn, shape, o, n in tr.fp.specs:
                r = go[o:o + n]
                errs[pn] = float((gh[o:o + n] - r).norm() / r.norm().clamp(min=1e-30))
            worst = sorted(errs.items(), key=lambda kv: -kv[1])[:3]
            print(json.dumps({"N": N, "B": a.B, "seed": seed, "env": a.env, "worst": worst}), flush=True)


if __name__ == "__main__":
    main()
