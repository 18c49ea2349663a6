"""Per-step kernel micro-benchmark (scan, ctrl_fwd, ctrl_node_bwd, ctrl_edge_bwd, node_combine)
on a realistic 1024-agent x 64-env rollout state.

usage: python scripts/micro_step.py [--so PATH] [--tag NAME] [--t STEP]
--so loads an alternative build of the extension (e.g. an ablation variant).
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
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--t", type=int, default=8)
ap.add_argument("--agents", type=int, default=1024)
ap.add_argument("--envs", type=int, default=64)
ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16", "fp16"])
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
from macbf_gnn_amd.parallel import DP  # noqa: E402

dev = torch.device("cuda")
cfg = C.TrainConfig(num_agents=args.agents, num_envs=args.envs, inner_loops=50, device="hip", seed=0,
                    dtype=args.dtype)
tr = Trainer(cfg, device=dev, dp=DP(device=dev))
eng = tr.engine
for _ in range(2):
    tr.train_step()                      # warm state (buffers hold a real rollout + backward)
torch.cuda.synchronize()
t = args.t
B, N, K, Nn = eng.B, eng.N, eng.K, eng.Nn
pw = eng.pw
rptr = eng.rptr[t * B:(t + 1) * B]
redges = eng.redges[t * B:(t + 1) * B]
valid = torch.ones(B, dtype=torch.uint8, device=dev)


def k_scan():
    native.scan(eng.S[t], eng.idx[t], eng.dang[t], eng.cnt[t], eng.safe[t], K=K, do_knn=True,
                do_safety=True, n_agents=N, prev_idx=eng.idx[t - 1])


def k_scan_nosort():
    native.scan(eng.S[t], eng.idx[t], eng.dang[t], eng.cnt[t], eng.safe[t], K=K, do_knn=True,
                do_safety=True, n_agents=N, prev_idx=eng.idx[t - 1], sort=False)


def k_scan_noprev():
    native.scan(eng.S[t], eng.idx[t], eng.dang[t], eng.cnt[t], eng.safe[t], K=K, do_knn=True,
                do_safety=True, n_agents=N)


def k_scan_nosafe():
    native.scan(eng.S[t], eng.idx[t], eng.dang[t], eng.cnt[t], eng.safe[t], K=K, do_knn=True,
                do_safety=False, n_agents=N, prev_idx=eng.idx[t - 1])


def k_scan_safeonly():
    native.scan(eng.S[t], None, None, None, eng.safe[t], K=K, do_knn=False, do_safety=True, n_agents=N)


def k_fwd():
    native.ctrl_fwd(eng.S[t], eng.G, eng.idx[t], pw.ctrl_w, pw.ctrl_off["ew1f"], pw.ctrl_off["nw1f"], pw.ctrl_v,
                    eng.A[t], eng.S[t + 1], eng.dist[t], eng.act[t], pooled=eng.pooled[t], argmax=eng.argmax[t],
                    prec=eng.prec)


def k_node():
    native.ctrl_node_bwd(eng.pooled[t], eng.S[t], eng.G, eng.A[t], eng.Gb[t + 1], valid, pw.ctrl_rm,
                         pw.node_rm_off, pw.ctrl_v, 1.0, eng.dP, eng.ego, eng.part_node, eng.nb_node,
                         act_cnt=eng.counts[2:3], prec=eng.prec)


def k_edge():
    native.ctrl_edge_bwd(eng.S[t], eng.idx[t], eng.argmax[t], eng.dP, pw.ctrl_w, pw.ctrl_off["ew1f"],
                         pw.ctrl_off["ew2tn"], eng.dEc[0], eng.part_edge, eng.nb_edge, prec=eng.prec)


def k_comb():
    native.node_combine(eng.dS[t], eng.ego, eng.dEc[0], rptr, redges, eng.Gb[t + 1], eng.Gb[t], K=K)


out = {"tag": args.tag, "dtype": args.dtype}
for name, fn in (("scan", k_scan), ("scan_nosort", k_scan_nosort), ("scan_noprev", k_scan_noprev), ("scan_nosafe", k_scan_nosafe), ("scan_safeonly", k_scan_safeonly), ("ctrl_fwd", k_fwd), ("node_bwd", k_node), ("edge_bwd", k_edge),
                 ("combine", k_comb)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    out[name] = round(e0.elapsed_time(e1) / args.iters * 1000, 1)   # us
print(json.dumps(out))
