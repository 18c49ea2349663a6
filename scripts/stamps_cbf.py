"""Phase clocks of the active-list CBF backward (diagnostics).

Runs warm-up training iterations at the headline config, captures the engine's cbf_bwd call,
re-runs it with a stamps buffer and prints the shader-clock cycles per chunk of each phase
(median over waves; the slowest wave's sum over its chunks in the last column), for the captured
active list and for all deduplicated evaluations.

    python scripts/stamps_cbf.py [--so PATH] [--envs 64]
"""
import argparse
import importlib.util
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = ["p0", "p1", "p2", "p3", "p4", "p5"]   # cbf_bwd: fwd A dH2 B dH1 CD; cbf_bwd16: fwd A dH2+dH1+dF BC;
#                                                 cbf_bwd_pw: fwd, head + image A + dW3, dH2 + dH1 + dF, image B + dW2 + dW1f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--so", default=None)
    ap.add_argument("--warm", type=int, default=2)
    ap.add_argument("--envs", type=int, default=64)
    a = ap.parse_args()
    import torch
    if a.so:
        spec = importlib.util.spec_from_file_location("macbf_gnn_amd._C", a.so)
        mod = importlib.util.module_from_spec(spec)
        sys.modules["macbf_gnn_amd._C"] = mod
        spec.loader.exec_module(mod)
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.ops import native

    dev = torch.device("cuda", 0)
    tr = Trainer(C.TrainConfig(num_agents=1024, num_envs=a.envs, inner_loops=50, device="hip", seed=0), device=dev)
    cap = {}
    orig = native.cbf_bwd

    def spy(*x, **k):
        if k.get("act") is not None or k.get("rec") is not None:
            cap["a"], cap["k"] = x, dict(k)
        return orig(*x, **k)

    native.cbf_bwd = spy
    for _ in range(a.warm):
        tr.train_step()
    torch.cuda.synchronize()
    native.cbf_bwd = orig
    x, k = cap["a"], cap["k"]
    nb = k["num_blocks"]
    nw = 8 if (k.get("rec") is not None or k.get("prec", None) not in ("fp32", None)) else 4
    nev = int(k["nev"][0])
    out = {}
    for mode in ("act", "all"):
        if mode == "all":
            sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
            from micro_cbfbwd_util import all_active
            all_active(x, k, nev, dev)
        st = torch.zeros(nb, nw, 8, dtype=torch.int64, device=dev)
        orig(*x, **k)
        orig(*x, stamps=st, **k)
        torch.cuda.synchronize()
        st = st.view(nb, nw, 8).double().cpu()
        busy_w = int((st[:, :, 7].sum(0) > 0).sum())    # the per-wave-dW kernel runs 4 waves
        st = st[:, :busy_w].reshape(-1, 8)
        st = st[st[:, 7] > 0]
        nch = st[:, 7].clamp(min=1)
        per = st[:, :6] / nch[:, None]
        med = per.median(dim=0).values
        tot = st[:, :6].sum(1)
        res = {p: round(float(v)) for p, v in zip(PHASES, med)}
        res["sum_per_chunk"] = round(float(med.sum()))
        # a chunk is 16 evaluations per wave: per CU 16 x (waves) evaluations per chunk time
        res["waves"] = busy_w
        res["cu_cycles_per_128_evals"] = round(float(med.sum()) * 128 / (16 * busy_w))
        res["chunks_per_wave"] = float(nch.median())
        res["slowest_wave_cycles"] = round(float(tot.max()))
        out[mode] = res
        print(mode, json.dumps(res))
    print(json.dumps({"nact": int(k["nact"][0]), "nev": nev, "blocks": nb, **out}))


if __name__ == "__main__":
    main()
