"""Compare the 16x16x32 x3 CBF backward (records) with the 32x32x16 x3 kernel (index list) on one
captured training call: per-section relative errors of the reduced weight-gradient slab and of
dE (diagnostics for csrc/cbf16.h).

    python scripts/check_cbf16.py [--agents 96 --envs 3]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SECTIONS = {"dW3": (0, 8192), "db3": (8192, 8256), "dW2": (8256, 16448), "db2": (16448, 16576),
            "dW1f": (16576, 18624), "dw4": (18624, 18688), "db4": (18688, 18689)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=96)
    ap.add_argument("--envs", type=int, default=3)
    ap.add_argument("--T", type=int, default=6)
    ap.add_argument("--so", default=None)
    a = ap.parse_args()
    import torch
    if a.so:
        import importlib.util
        spec = importlib.util.spec_from_file_location("macbf_gnn_amd._C", a.so)
        mod = importlib.util.module_from_spec(spec)
        sys.modules["macbf_gnn_amd._C"] = mod
        spec.loader.exec_module(mod)
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.ops import native

    dev = torch.device("cuda", 0)
    tr = Trainer(C.TrainConfig(num_agents=a.agents, num_envs=a.envs, inner_loops=a.T, device="hip", seed=0),
                 device=dev)
    cap = {}
    orig = native.cbf_bwd

    def spy(*x, **k):
        if k.get("rec") is not None:
            cap["a"], cap["k"] = x, dict(k)
        return orig(*x, **k)

    native.cbf_bwd = spy
    tr.train_step()
    torch.cuda.synchronize()
    native.cbf_bwd = orig
    x, k = cap["a"], cap["k"]
    nact = int(k["nact"][0])
    rec = k["rec"]
    dE = k["dE"]
    part = k["partial"]
    outs = {}
    for mode in ("new", "old"):
        dE.zero_()
        part.zero_()
        kk = dict(k)
        if mode == "old":
            act = torch.zeros(rec.shape[0], dtype=torch.int32, device=dev)
            act[:nact] = rec[:nact, 0]
            kk.pop("rec"); kk.pop("wrm16"); kk.pop("w16")
            kk["act"] = act
        dbg = torch.zeros(3 * nact + 3, dtype=torch.float32, device=dev)
        if mode == "new" and os.environ.get("CHK_DBG", "0") == "1":
            dbg = torch.zeros(3 * nact + 3, dtype=torch.float32, device=dev)
            kk["dbg"] = dbg
        orig(*x, **kk)
        torch.cuda.synchronize()
        outs[mode] = (dE.clone(), part.double().sum(0))
    res = {"nact": nact}
    for name, (lo, hi) in SECTIONS.items():
        n, o = outs["new"][1][lo:hi], outs["old"][1][lo:hi]
        res[name] = float((n - o).norm() / o.norm().clamp(min=1e-30))
    u = rec[:nact, 0].long()
    dn, do = outs["new"][0].view(-1, dE.shape[-1])[u], outs["old"][0].view(-1, dE.shape[-1])[u]
    res["dE"] = float((dn - do).norm() / do.norm().clamp(min=1e-30))
    bad = ((dn - do).norm(dim=1) > 1e-3 * do.norm(dim=1) + 1e-9).nonzero().flatten()
    res["dE_bad_rows"] = int(bad.numel())
    res["dE_bad_first"] = [int(v) for v in bad[:16]]
    res["dE_bad_u"] = [int(u[v]) for v in bad[:8]]
    res["dE_bad_pass"] = [int(rec[v, 1]) < 0 for v in bad[:8].tolist()]
    # independent fp64 reference of dE for the first bad rows (and a few good ones)
    S = x[0]
    idx = x[1]
    T, B, N, K = idx.shape
    E = idx.numel()
    prm = {pn: tr.fp.flat[o:o + n].view(shape).double().cpu() for (m, pn, shape, o, n) in tr.fp.specs}
    W1, b1 = prm["cbf_net.0.weight"].reshape(64, -1), prm["cbf_net.0.bias"]
    W2, b2 = prm["cbf_net.2.weight"].reshape(128, -1), prm["cbf_net.2.bias"]
    W3, b3 = prm["cbf_net.4.weight"].reshape(64, -1), prm["cbf_net.4.bias"]
    W4 = prm["cbf_net.6.weight"].reshape(1, -1)
    rows = torch.cat([bad[:24].cpu(), torch.arange(0, min(nact, 8))])
    errs = []
    for v in rows.tolist():
        u_, y, j, dhb = [int(q) for q in rec[v].tolist()]
        pas = 1 if y < 0 else 0
        e = y & 0x7FFFFFFF
        ik = e // K
        tb, i = divmod(ik, N)
        t, b = divmod(tb, B)
        si = S[t + pas, b, i, :4].double().cpu()
        sj = S[t + pas, b, j, :4].double().cpu()
        dhv = torch.tensor([dhb], dtype=torch.int32).view(torch.float32).double().item()
        r = (si - sj).clone().requires_grad_(True)
        d = torch.sqrt((r[:2] ** 2).sum() + float(C.CBF_DIST_EPS_COORD * 2))
        feat = torch.cat([r, torch.tensor([1.0 if i == j else 0.0], dtype=torch.float64), (d - C.DIST_MIN_THRES).view(1)])
        h1 = torch.relu(W1 @ feat + b1)
        h2 = torch.relu(W2 @ h1 + b2)
        h3 = torch.relu(W3 @ h2 + b3)
        h = (W4 @ h3).sum()
        (gr,) = torch.autograd.grad(h * dhv, r)
        dv3 = dbg[3 * v: 3 * v + 3].double().cpu().tolist()
        sums = {"h1": [dv3[0], float(h1.sum())], "h2": [dv3[1], float(h2.sum())], "h": [dv3[2], float(h)]}
        ref = gr if i != j else torch.zeros(4, dtype=torch.float64)
        dn_ = outs["new"][0].view(-1, dE.shape[-1])[u_].double().cpu()
        do_ = outs["old"][0].view(-1, dE.shape[-1])[u_].double().cpu()
        errs.append({"v": v, "pass": pas, "self": i == j, "n": v % 16, "wave": (v // 16) % 8,
                     "e_new": float((dn_ - ref).norm() / ref.norm().clamp(min=1e-30)),
                     "e_old": float((do_ - ref).norm() / ref.norm().clamp(min=1e-30)), **sums})
    for q in errs:
        print(json.dumps(q))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
