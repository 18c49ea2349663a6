"""Micro-benchmark of the deduplicated CBF kernels (the default training path) at 1024 agents x
64 envs: one training iteration fills the evaluation list, the upstream gradients and the
active list; then cbf_hfwd over the whole list and cbf_bwd over the active list are re-launched
with the same arguments and timed (both are idempotent: they only write h / dE / the slabs).

usage: python scripts/micro_cbf_dedup.py [--dtype fp32|bf16] [--tag NAME]
Set MACBF_EXT=path/_C.so to time a variant build (scripts/build_variants.sh cbf_x3 ...).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--tag", default="base")
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16", "fp16"])
ap.add_argument("--train_iters", type=int, default=1)
args = ap.parse_args()
import torch  # noqa: E402

from macbf_gnn_amd import config as C  # noqa: E402
from macbf_gnn_amd.engine import Trainer  # noqa: E402
from macbf_gnn_amd.ops import native  # noqa: E402
from macbf_gnn_amd.parallel import DP  # noqa: E402

dev = torch.device("cuda")
cfg = C.TrainConfig(num_agents=1024, num_envs=64, inner_loops=50, device="hip", seed=0, dtype=args.dtype)
tr = Trainer(cfg, device=dev, dp=DP(device=dev))
for _ in range(args.train_iters):
    st = tr.train_step()
torch.cuda.synchronize()
eng = tr.engine
T = int(float(st["T"]))
B, N, K, W = eng.B, eng.N, eng.K, eng.W
E = T * B * N * K
pw = eng.pw
S, idx = eng.S[: T + 1], eng.idx[:T]
src, nev = eng.src[: 2 * E], eng.nev_dev
dh = eng.dhbuf[: 2 * E]
act, nact = eng.act_list[: 2 * E], eng.nact_dev
nbb = native.cbf_bwd_grid(2 * E, dev)
part = eng._buf(eng._part_cbf, nbb, native.CBF_PARTIAL)
dE = eng.dE[: 2 * E * W].view(2, T, B, N, K, W)
hb, hm = eng.hbuf[: 2 * E].clone(), eng.hmask[: 2 * E].clone()


def bwd():
    native.cbf_bwd(S, idx, dh.view(2, T, B, N, K), pw.cbf_w, pw.cbf_off["w1f"], pw.cbf_rm, pw.cbf_v, passes=2,
                   dE=dE, partial=part, num_blocks=nbb, idx1=idx, src=src, nev=nev, act=act, nact=nact,
                   prec=eng.prec)


def hfwd():
    native.cbf_hfwd(S, idx, idx, src, nev, pw.cbf_w, pw.cbf_off["w1f"], pw.cbf_rm, pw.cbf_v, hb, hm, u_begin=0,
                    prec=eng.prec)


def timeit(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / args.iters


ms_b = timeit(bwd)
ms_h = timeit(hfwd)
n_ev, n_act = int(nev.view(-1)[0].item()), int(nact.view(-1)[0].item())
print(json.dumps({"tag": args.tag, "dtype": args.dtype, "T": T, "evals": n_ev, "active": n_act,
                  "cbf_bwd_ms": round(ms_b, 4), "cbf_hfwd_all_ms": round(ms_h, 4),
                  "bwd_Mevals_per_s": round(n_act / ms_b / 1e3, 1),
                  "slab_checksum": float(part.double().sum())}))
