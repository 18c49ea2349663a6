"""Host-side issue time of the training step's phases at a small config (diagnostics): wraps the
HIP engine's rollout / counts / backward and the trainer's optimizer step with host timers and
reports the mean host milliseconds per iteration next to the wall time per iteration.

    python scripts/host_overhead.py [--agents 32 --envs 1 --iters 40]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=32)
    ap.add_argument("--envs", type=int, default=1)
    ap.add_argument("--iters", type=int, default=40)
    a = ap.parse_args()
    import torch
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.engine.hip_engine import HipEngine
    dev = torch.device("cuda")
    cfg = C.TrainConfig(num_agents=a.agents, num_envs=a.envs, device="hip", seed=0, display_steps=10 ** 9,
                        save_steps=10 ** 9)
    tr = Trainer(cfg)
    acc = {}

    def wrap(obj, name, key):
        f = getattr(obj, name)

        def g(*args, **kw):
            t0 = time.perf_counter()
            r = f(*args, **kw)
            acc[key] = acc.get(key, 0.0) + time.perf_counter() - t0
            return r
        setattr(obj, name, g)
    eng = tr.engine
    for name in ("rollout", "_counts", "_backward", "_stats"):
        wrap(eng, name, name)
    for _ in range(10):
        tr.train_step()
    torch.cuda.synchronize()
    acc.clear()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        tr.train_step()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.iters * 1e3
    out = {"agents": a.agents, "envs": a.envs, "wall_ms": round(wall, 3)}
    out.update({k: round(v / a.iters * 1e3, 3) for k, v in acc.items()})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
