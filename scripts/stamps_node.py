"""Phase clocks of the node backward (diagnostics): runs two training steps at the given config,
then one ctrl_node_bwd call with the stamps buffer and prints, per phase, the median over
workgroups of the slowest wave's shader-clock delta (cycles). Default: the cooperative 32-agent
kernel, whose stamps are compiled only into a diagnostics build (MACBF_EXT=alt_so/stamps/_C.so from
scripts/build_variant.sh stamps ctrl_x3 "-DMB_DIAG=1"); --node16: the 16x16x32 kernel
(csrc/node16.h, 128-agent chunks, 8 waves; its stamps instantiation ships in every build).

    python scripts/stamps_node.py [--agents 1024 --envs 8] [--node16 --envs 64]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = ["start", "weights", "loads", "L1", "L2", "L3", "L4+gain", "dY3", "S4/S3+dY2", "S2+dY1",
          "S1 stage", "S1", "dP", "chunk end", "slab"]
PHASES16 = ["start", "weights", "loads+combine", "forward", "gain+dY3", "stage1", "dY2+dY1", "stage2", "stage3",
            "dP ego tile", "dP tiles 0-3", "dP tiles 4-7", "-", "chunk end", "slab"]
ORDER16 = [2, 3, 4, 5, 6, 7, 8, 10, 11, 9, 12, 13, 14]   # slots in time order (10, 11 inside the dP loop)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=1024)
    ap.add_argument("--envs", type=int, default=8)
    ap.add_argument("--t", type=int, default=4)
    ap.add_argument("--node16", action="store_true")
    ap.add_argument("--blocks", type=int, default=0, help="workgroups (default: one per chunk); fewer -> "
                    "each runs several chunks and the LAST (warm instruction cache) chunk is reported")
    a = ap.parse_args()
    import torch
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.ops import native
    from macbf_gnn_amd.parallel import DP
    dev = torch.device("cuda")
    cfg = C.TrainConfig(num_agents=a.agents, num_envs=a.envs, inner_loops=50, device="hip", seed=0)
    tr = Trainer(cfg, device=dev, dp=DP(device=dev))
    for _ in range(2):
        tr.train_step()
    torch.cuda.synchronize()
    eng, pw, t = tr.engine, tr.engine.pw, a.t
    valid = torch.ones(eng.B, dtype=torch.uint8, device=dev)
    nb = a.blocks or eng.nb_node
    NW = 8 if a.node16 else 4
    st = torch.zeros(nb, NW, 16, dtype=torch.int64, device=dev)
    part = eng.part_node[:nb]
    for rep in range(3):
        st.zero_()
        native.ctrl_node_bwd(eng.pooled[t], eng.S[t], eng.G, eng.A[t], eng.Gb[t + 1], valid, pw.ctrl_rm,
                             pw.node_rm_off, pw.ctrl_v, 1.0, eng.dP, eng.ego, part, nb,
                             act_cnt=eng.counts[2:3], prec=eng.prec, stamps=st, chunk=128 if a.node16 else 32,
                             wrm16=pw.node_rm16 if a.node16 else None)
        torch.cuda.synchronize()
    s = st.cpu()
    used = s[:, 0, 0] > 0
    s = s[used]
    t0 = s[:, :, 0].min(dim=1).values                      # workgroup start (earliest wave)
    out = {"agents": a.agents, "envs": a.envs, "workgroups": int(used.sum())}
    prev = t0
    rows = []
    w1 = s[:, :, 1].max(dim=1).values
    rows.append(("weights", float((w1 - t0).float().median()), float((w1 - t0).float().max())))
    prev = s[:, :, 15].max(dim=1).values                   # (last) chunk start
    rows.append(("to chunk start", float((prev - w1).float().median()), float((prev - w1).float().max())))
    names = PHASES16 if a.node16 else PHASES
    for k in (ORDER16 if a.node16 else range(2, 15)):
        if names[k] == "-":
            continue
        tk = s[:, :, k].max(dim=1).values                  # slowest wave reaches phase end
        d = (tk - prev).float()
        rows.append((names[k], float(d.median()), float(d.max())))
        prev = tk
    total = (s[:, :, 14].max(dim=1).values - t0).float()
    out["total_median_cycles"] = float(total.median())
    out["phases_median_cycles"] = {n: round(m) for n, m, _ in rows}
    print(json.dumps(out))
    for n, m, x in rows:
        print(f"  {n:16s} median {m:8.0f} cyc   max {x:8.0f}")


if __name__ == "__main__":
    main()
