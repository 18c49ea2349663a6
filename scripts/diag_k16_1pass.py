"""Diagnostics of the 16x16x32 backward kernels in the 1-pass (bf16 / fp16) builds: capture one CBF
backward call (record list) and one BPTT edge backward call of a real training step, re-run the
16x16x32 kernel on the captured inputs and compare with the float64 oracles of ops/selfcheck
(relative row error statistics, NaN counts) and, for the edge kernel, with the 32x32x16 kernel on
the same inputs (dEc rows and reduced weight-gradient slabs).

    python scripts/diag_k16_1pass.py [--dtype bf16] [--agents 32 --envs 2 --T 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--agents", type=int, default=32)
    ap.add_argument("--envs", type=int, default=2)
    ap.add_argument("--T", type=int, default=5)
    a = ap.parse_args()
    os.environ["MACBF_NATIVE_BPTT"] = "0"      # Python launch loop: the spies see the calls
    os.environ["MACBF_BWD_FUSED"] = "0"
    import torch
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.ops import layout as L
    from macbf_gnn_amd.ops import native
    from macbf_gnn_amd.ops.selfcheck import cbf_record_oracle, edge_oracle
    dev = torch.device("cuda", 0)
    tr = Trainer(C.TrainConfig(device="hip", seed=0, dtype=a.dtype, num_agents=a.agents, num_envs=a.envs,
                               inner_loops=a.T, early_stop=False), device=dev)
    eng = tr.engine
    cap = {"cbf": None, "edge": []}
    o_cbf, o_edge = native.cbf_bwd, native.ctrl_edge_bwd

    def spy_cbf(*x, **k):
        if k.get("rec") is not None:
            cap["cbf"] = (x, dict(k))
        return o_cbf(*x, **k)

    def spy_edge(*x, **k):
        if not k.get("_defer"):
            cap["edge"].append((x, dict(k)))
        return o_edge(*x, **k)

    native.cbf_bwd, native.ctrl_edge_bwd = spy_cbf, spy_edge
    flat0 = tr.fp.flat.clone()
    tr.train_step()
    torch.cuda.synchronize()
    native.cbf_bwd, native.ctrl_edge_bwd = o_cbf, o_edge
    tr.fp.flat.copy_(flat0)
    eng.after_update()
    out = {"dtype": a.dtype, "cbf16": eng.cbf16, "eb16": eng.eb16_w is not None}
    params = lambda mod: {pn: tr.fp.flat[o:o + n].view(shape).detach().double()
                          for m, pn, shape, o, n in tr.fp.specs if m == mod}

    def stats(got, ref):
        err = (got - ref).norm(dim=-1)
        rn = ref.norm(dim=-1)
        rel = err / (rn + 1e-12)
        nz = rn > 0
        return {"rows": int(got.shape[0]), "nan_rows": int((~torch.isfinite(got)).any(-1).sum()),
                "rel_median": float(rel[nz].median()) if nz.any() else 0.0,
                "rel_p99": float(rel[nz].quantile(0.99)) if nz.sum() > 1 else 0.0,
                "rows_rel_gt_0.1": int((rel[nz] > 0.1).sum()),
                "total_rel": float(err.norm() / (rn.norm() + 1e-30))}

    if cap["cbf"] is not None:
        x, k = cap["cbf"]
        nact = int(k["nact"][0])
        rec = k["rec"][:nact].clone()
        k["dE"].zero_()
        k["partial"].fill_(float("nan"))
        o_cbf(*x, **k)
        torch.cuda.synchronize()
        S, idx = x[0], x[1]
        T, B, N, K = idx.shape
        W = k["dE"].shape[-1]
        ref, tie, ref_dw, scale, rscale = cbf_record_oracle(params("cbf"), S, rec, T, B, N, K, tr.cfg.dim)
        got = native.from_records(k["dE"].view(-1, W)[rec[:, 0].long()]).double()
        out["cbf_dE"] = stats(got, ref)
        part = k["partial"]
        out["cbf_partial_nan_rows"] = int((~torch.isfinite(part)).any(-1).sum())
        out["cbf_partial_rows"] = int(part.shape[0])
    if cap["edge"]:
        x, k = cap["edge"][len(cap["edge"]) // 2]
        res = {}
        for name, w16 in (("k16", k.get("w16")), ("k32", None)):
            kk = dict(k)
            kk["init"] = True
            kk["w16"] = w16
            kk["partial"] = torch.full_like(k["partial"], float("nan"))
            kk["dEc"] = torch.zeros_like(k["dEc"])
            o_edge(*x, **kk)
            torch.cuda.synchronize()
            sm, dm = L.ctrl_edge_grad_map({pn: o for (m, pn, s, o, n) in tr.fp.specs}, tr.cfg.dim)
            red = kk["partial"].double().sum(0)
            g = torch.zeros_like(tr.fp.flat, dtype=torch.float64)
            g.index_add_(0, torch.as_tensor(dm, device=dev), red.index_select(0, torch.as_tensor(sm, device=dev)))
            res[name] = (native.from_records(kk["dEc"]).double(), g, int((~torch.isfinite(kk["partial"])).any(-1).sum()))
        S, idx, am, dP = k["S"], k["idx"], k["argmax"], k["dP"]
        B, N, K = idx.shape
        D = tr.cfg.dim
        # 1-pass rows (128 wide): the oracle reads [hi | lo]
        dP2 = torch.cat([dP, torch.zeros_like(dP)], -1) if dP.shape[-1] == 128 else dP
        ref, tie, ref_dw, scale, rscale = edge_oracle(params("controller"), S, idx, am, dP2, N, D)
        for name, (dEc, g, nanrows) in res.items():
            out[f"edge_{name}_dEc"] = stats(dEc.reshape(-1, 2 * D), ref.reshape(-1, 2 * D))
            out[f"edge_{name}_partial_nan_rows"] = nanrows
            for m, pn, shape, o, n in tr.fp.specs:
                if pn in ref_dw:
                    r = ref_dw[pn].reshape(-1)
                    out[f"edge_{name}_{pn}_rel"] = float((g[o:o + n] - r).norm() / (r.norm() + 1e-30))
        out["edge_k16_vs_k32_dEc"] = float((res["k16"][0] - res["k32"][0]).norm() / (res["k32"][0].norm() + 1e-30))
        out["edge_k16_vs_k32_grad"] = float((res["k16"][1] - res["k32"][1]).norm() / (res["k32"][1].norm() + 1e-30))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
