"""Micro-benchmark of the deduplicated active-list CBF backward (the training default).

Runs warm-up training iterations at the headline config, captures the engine's cbf_bwd call of
the last one and re-times it: (a) on the captured active list, (b) on ALL deduplicated
evaluations (the mid-training regime, ~94 % active). Prints one JSON line with both timings,
the per-evaluation cost and a checksum of the weight-gradient slabs (bit-identity across builds).

usage: python scripts/micro_cbfbwd.py [--so PATH] [--tag NAME] [--iters 10] [--warm 2]
"""
import argparse
import importlib.util
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

ap = argparse.ArgumentParser()
ap.add_argument("--so", default=None)
ap.add_argument("--tag", default="base")
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--warm", type=int, default=2)
ap.add_argument("--agents", type=int, default=1024)
ap.add_argument("--envs", type=int, default=64)
args = ap.parse_args()
import torch  # noqa: E402

if args.so:
    spec = importlib.util.spec_from_file_location("macbf_gnn_amd._C", args.so)
    mod = importlib.util.module_from_spec(spec)
    sys.modules["macbf_gnn_amd._C"] = mod
    spec.loader.exec_module(mod)

from macbf_gnn_amd import config as C  # noqa: E402
from macbf_gnn_amd.engine import Trainer  # noqa: E402
from macbf_gnn_amd.ops import native  # noqa: E402
from micro_cbfbwd_util import all_active  # noqa: E402

dev = torch.device("cuda", 0)
cfg = C.TrainConfig(num_agents=args.agents, num_envs=args.envs, inner_loops=50, device="hip", seed=0)
tr = Trainer(cfg, device=dev)
cap = {}
_orig = native.cbf_bwd


def _spy(*a, **k):
    if k.get("act") is not None or k.get("rec") is not None:
        cap["a"], cap["k"] = a, dict(k)
    return _orig(*a, **k)


native.cbf_bwd = _spy
for _ in range(args.warm):
    tr.train_step()
torch.cuda.synchronize()
native.cbf_bwd = _orig
assert "a" in cap, "no active-list cbf_bwd call captured (dedup path off?)"
a, k = cap["a"], cap["k"]
nev = int(k["nev"][0])
nact = int(k["nact"][0])


def timed():
    for _ in range(2):
        _orig(*a, **k)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        _orig(*a, **k)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / args.iters, float(k["partial"].double().sum())


ms_act, chk_act = timed()
# all deduplicated evaluations active (dh kept as is: zeros only change the arithmetic values)
all_active(a, k, nev, dev)
ms_all, chk_all = timed()
print(json.dumps({"tag": args.tag, "nev": nev, "nact": nact, "ms_act": round(ms_act, 4),
                  "ns_per_act": round(ms_act * 1e6 / max(nact, 1), 4), "ms_all": round(ms_all, 4),
                  "ns_per_eval_all": round(ms_all * 1e6 / nev, 4), "chk_act": chk_act, "chk_all": chk_all}))
