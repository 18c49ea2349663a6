"""Scan micro-benchmark on realistic rollout states: times cell_sort+scan variants."""
import json
import sys
import time

import torch

import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from macbf_gnn_amd import config as C  # noqa: E402
from macbf_gnn_amd.engine import Trainer  # noqa: E402
from macbf_gnn_amd.parallel import DP  # noqa: E402
from macbf_gnn_amd.ops import native  # noqa: E402

dev = torch.device("cuda")
B, N = 64, int(sys.argv[1]) if len(sys.argv) > 1 else 1024
cfg = C.TrainConfig(num_agents=N, num_envs=B, inner_loops=20, device="hip", early_stop=False)
tr = Trainer(cfg, device=dev, dp=DP(device=dev))
s0, g, _ = tr.sample()
tr.engine.rollout(s0, g)
S = tr.engine.S[10].contiguous()
K = min(N, C.TOP_K)
idx = torch.empty(B, N, K, dtype=torch.int32, device=dev)
dang = torch.empty(B, N, K, dtype=torch.uint8, device=dev)
cnt = torch.zeros(B, 2, device=dev)
safe = torch.zeros(B, device=dev)
res = {}
for name, kw in (("full", dict(do_knn=True, do_safety=True)), ("knn", dict(do_knn=True, do_safety=False)),
                 ("safety", dict(do_knn=False, do_safety=True))):
    a = (idx, dang, cnt, safe) if kw["do_knn"] else (None, None, None, safe)
    for _ in range(5):
        native.scan(S, *a, K=K, **kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        native.scan(S, *a, K=K, **kw)
    e1.record()
    torch.cuda.synchronize()
    res[name] = e0.elapsed_time(e1) / 50 * 1000
print(json.dumps({"N": N, "B": B, "us_per_call": res}))
