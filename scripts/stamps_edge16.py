"""Phase clocks of the 16x16x32 controller edge backward (csrc/ctrl16.h, diagnostics): runs two
training steps at the given config, then the engine's edge backward call of step --t with the
stamps buffer (the kernel's ST instantiation; the production kernel has no stamps) and prints, per
phase, the cycles per 16-edge tile (median and max over waves), the tiles per wave and the
slowest wave's loop total (phases: csrc/ctrl16.h).

    python scripts/stamps_edge16.py [--agents 1024 --envs 64 --t 4 --dtype fp32]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = ["load issue", "F", "layer 1", "dZ zero fill", "routing", "dH1", "dF+dEc", "H1 store", "barrier 1",
          "S1", "barrier 2", "S2 stores", "S2 contraction"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=1024)
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--t", type=int, default=4)
    ap.add_argument("--dtype", default="fp32")
    a = ap.parse_args()
    os.environ.setdefault("MACBF_SELFCHECK", "0")
    import torch
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.ops import native
    dev = torch.device("cuda", 0)
    cfg = C.TrainConfig(num_agents=a.agents, num_envs=a.envs, inner_loops=50, device="hip", seed=0, dtype=a.dtype)
    tr = Trainer(cfg, device=dev)
    eng = tr.engine
    if eng.eb16_w is None:
        raise SystemExit("this configuration does not run the 16x16x32 edge backward (MACBF_EB16)")
    for _ in range(2):
        tr.train_step()
    torch.cuda.synchronize()
    pw, t, nb = eng.pw, a.t, eng.nb_edge
    st = torch.zeros(nb, 8, 16, dtype=torch.int64, device=dev)
    part = torch.zeros(nb, native.CTRL_EDGE_PARTIAL, device=dev)
    dEc = torch.zeros_like(eng.dEc[0])
    for rep in range(3):
        st.zero_()
        native.ctrl_edge_bwd(eng.S[t], eng.idx[t], eng.argmax[t], eng.dP, pw.ctrl_w, pw.ctrl_off["ew1f"],
                             pw.ctrl_off["ew2tn"], dEc, part, nb, prec=eng.prec, init=True, w16=eng.eb16_w, stamps=st)
        torch.cuda.synchronize()
    s = st.cpu().reshape(-1, 16).double()
    s = s[s[:, 15] > 0]
    tiles = s[:, 15]
    out = {"agents": a.agents, "envs": a.envs, "dtype": a.dtype, "workgroups": nb,
           "tiles_per_wave_median": float(tiles.median())}
    per = s[:, :13] / tiles.unsqueeze(1)
    rows = []
    for k, name in enumerate(PHASES):
        rows.append((name, float(per[:, k].median()), float(per[:, k].max())))
    tot = s[:, :13].sum(1)
    out["loop_cycles_per_tile_median"] = float((tot / tiles).median())
    out["slowest_wave_loop_cycles"] = float(tot.max())
    out["phases_cycles_per_tile_median"] = {n: round(m) for n, m, _ in rows}
    print(json.dumps(out))
    for n, m, x in rows:
        print(f"  {n:14s} median {m:8.0f} cyc/tile   max {x:8.0f}")


if __name__ == "__main__":
    main()
