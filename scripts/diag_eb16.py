"""Rows of the 16x16x32 edge backward that disagree with the float64 oracle (diagnostics for
tests/test_gpu_oracle16.py): per bad edge its (b, i, k), neighbour j, distance, mask, the number of
max-pool features routed to it, kernel row, oracle row and row scale.

    python scripts/diag_eb16.py [--agents 96 --envs 3]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


class _MP:
    def setenv(self, k, v):
        os.environ[k] = v

    def setattr(self, obj, name, val):
        setattr(obj, name, val)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=96)
    ap.add_argument("--envs", type=int, default=3)
    a = ap.parse_args()
    import torch
    import test_gpu_oracle16 as T
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd.ops import native
    tr, orig, (args, k) = T._capture_edge(_MP(), num_agents=a.agents, num_envs=a.envs, inner_loops=6)
    kk = dict(k)
    kk["init"] = True
    kk["partial"] = torch.zeros_like(k["partial"])
    kk["dEc"] = torch.zeros_like(k["dEc"])
    orig(*args, **kk)
    torch.cuda.synchronize()
    S, idx, argmax, dP = kk["S"], kk["idx"], kk["argmax"], kk["dP"]
    B, N, K = idx.shape
    D = tr.cfg.dim
    ref, tie, _, _, rscale = T.edge_oracle(T._params(tr, "controller"), S, idx, argmax, dP, N, D)
    got = native.from_records(kk["dEc"]).double()
    err = (got - ref).norm(dim=-1)
    tol = T.ROW_TOL * ref.norm(dim=-1) + T.ABS_TOL * rscale.norm(dim=-1) + 1e-30
    bad = (err > tol) & ~tie
    Sf = native.from_records(S).double()
    print("bad", int(bad.sum()), "of", bad.numel())
    for b, i, kq in bad.nonzero().tolist()[:20]:
        j = int(idx[b, i, kq])
        d = float((Sf[b, i, :D] - Sf[b, j, :D]).norm())
        routed = int((argmax[b, i].long() == kq).sum())
        print(f"b={b} i={i} k={kq} j={j} d={d:.6f} mask={d < C.OBS_RADIUS} routed={routed} "
              f"got={got[b, i, kq].tolist()} ref={ref[b, i, kq].tolist()} scale={rscale[b, i, kq].norm():.3e}")


if __name__ == "__main__":
    main()
