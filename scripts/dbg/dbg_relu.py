"""Debug: are the fp32 (x3) CBF-backward outliers relu boundary flips? Near-zero pre-activations
(float64) of the edges between the worst agent pairs."""
import sys
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import torch
from macbf_gnn_amd import config as C
from macbf_gnn_amd import oracle as O
import test_gpu_fp32 as F
F.DEV = torch.device("cpu")
T, B, N = 3, 2, 40
ctrl, cbf, fp, pw = F._nets(2)
K = min(N, C.TOP_K)
S = F._states((T + 1, B), N, seed=7, dens=0.6).contiguous().double()
idx = torch.stack([O.knn_idx(S[t].float(), K) for t in range(T)]).long()
p = {k: v.detach().double() for k, v in cbf.params_dict().items()}
for ps in range(2):
    x, mask = O.cbf_features(S[ps:ps + T], idx)
    z = x
    mins = []
    for i in (0, 2, 4):
        W = p[f"cbf_net.{i}.weight"].reshape(p[f"cbf_net.{i}.weight"].shape[0], -1)
        pre = z @ W.t() + p[f"cbf_net.{i}.bias"]
        sc = (z.abs() @ W.abs().t() + p[f"cbf_net.{i}.bias"].abs())      # sum |terms|
        mins.append((pre.abs() / sc).min(-1).values)                     # per edge: closest relu to 0
        z = torch.relu(pre)
    m = torch.stack(mins, -1).min(-1).values       # (T,B,N,K)
    for (t, b, i, j) in [(1, 0, 15, 28), (1, 0, 28, 15), (3, 1, 20, 31), (3, 1, 31, 20), (0, 0, 15, 28), (0, 0, 28, 15), (2, 1, 20, 31), (2, 1, 31, 20)]:
        tt = t - ps
        if not (0 <= tt < T):
            continue
        ks = (idx[tt, b, i] == j).nonzero().flatten().tolist()
        for k in ks:
            print(f"pass {ps} step {tt} b {b} edge {i}->{j} slot {k}: min |pre|/sum|terms| = {m[tt, b, i, k].item():.2e}  mask {mask[tt,b,i,k].item()}")
    print(f"pass {ps}: edges with a relu pre-activation within 1e-5 / 1e-4 of zero (relative):",
          int((m < 1e-5).sum()), int((m < 1e-4).sum()), "of", m.numel())
