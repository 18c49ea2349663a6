"""CBF training-kernel micro-benchmark on a realistic 1024-agent x 64-env rollout.

usage: python scripts/micro_cbf.py [--so PATH] [--tag NAME]
--so loads an alternative build of the extension (e.g. an experiment variant compiled by
scripts/build_variants.sh cbf) in place of macbf_gnn_amd._C before anything imports it.
"""
import argparse
import importlib.util
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--so", default=None)
ap.add_argument("--tag", default="base")
ap.add_argument("--iters", type=int, default=20)
args = ap.parse_args()
import torch  # noqa: E402  (HIP runtime initialised by torch before the extension loads)

if args.so:
    spec = importlib.util.spec_from_file_location("macbf_gnn_amd._C", args.so)
    mod = importlib.util.module_from_spec(spec)
    sys.modules["macbf_gnn_amd._C"] = mod
    spec.loader.exec_module(mod)

from macbf_gnn_amd import config as C  # noqa: E402
from macbf_gnn_amd.engine import Trainer  # noqa: E402
from macbf_gnn_amd.ops import native  # noqa: E402
from macbf_gnn_amd.parallel import DP  # noqa: E402

dev = torch.device("cuda")
cfg = C.TrainConfig(num_agents=1024, num_envs=64, inner_loops=50, device="hip", seed=0)
tr = Trainer(cfg, device=dev, dp=DP(device=dev))
eng = tr.engine
s0, g, obs = tr.sample()
T = eng.rollout(s0, g, obs)
B, N, K, W = eng.B, eng.N, eng.K, eng.W
done = (eng.dist[:T].double() / native.FX_DIST / N) < C.DIST_MIN_CHECK
di = done.to(torch.int32)
valid = ((torch.cumsum(di, 0) - di) == 0).to(torch.uint8).contiguous()
vf = valid.float()
eng.counts[0] = (eng.cnt[:T, :, 0] * vf).sum()
eng.counts[1] = (eng.cnt[:T, :, 1] * vf).sum()
eng.counts[2] = vf.sum() * N
E = T * B * N * K
nbb = native.cbf_bwd_grid(2 * E, dev)
part = torch.zeros(nbb, native.CBF_PARTIAL, device=dev)
dE = eng.dE[: 2 * E * W].view(2, T, B, N, K, W)
pw = eng.pw


def run():
    native.cbf_bwd(eng.S[: T + 1], eng.idx[:T], None, pw.cbf_w, pw.cbf_off["w1f"], pw.cbf_rm, pw.cbf_v, passes=2,
                   dE=dE, partial=part, num_blocks=nbb, fused=True, dang=eng.dang[:T], valid=valid,
                   counts=eng.counts)


for _ in range(3):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(args.iters):
    run()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / args.iters
chk = float(part.double().sum())
print(json.dumps({"tag": args.tag, "T": T, "edges": E, "blocks": nbb, "ms": round(ms, 4),
                  "Medge_evals_per_s": round(2 * E / ms / 1e3, 1), "slab_checksum": chk}))
