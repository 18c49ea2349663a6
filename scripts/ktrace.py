"""Per-iteration timeline summary from a rocprofv3 kernel_trace.csv: iteration wall time
(scenario_kernel to scenario_kernel), busy time, and the time between the rollout's last
controller step and the first BPTT kernel (the CBF phase), per iteration."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
its = [i for i, r in enumerate(rows) if "scenario_kernel" in r["Kernel_Name"]]
for a, b in zip(its[:-1], its[1:]):
    seg = rows[a:b]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    busy, last = 0, t0
    for r in seg:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += max(0, en - max(st, last))
        last = max(last, en)
    fwd = [i for i, r in enumerate(seg) if "ctrl_fwd" in r["Kernel_Name"]]
    nb = [i for i, r in enumerate(seg) if "ctrl_node_bwd" in r["Kernel_Name"]]
    roll = (int(seg[fwd[-1]]["End_Timestamp"]) - t0) / 1e6 if fwd else 0
    cbf = (int(seg[nb[0]]["Start_Timestamp"]) - int(seg[fwd[-1]]["End_Timestamp"])) / 1e6 if fwd and nb else 0
    bptt = (int(seg[nb[-1]]["End_Timestamp"]) - int(seg[nb[0]]["Start_Timestamp"])) / 1e6 if nb else 0
    print(f"iter wall {(t1 - t0) / 1e6:.3f} ms busy {busy / 1e6:.3f}  rollout {roll:.3f}  cbf {cbf:.3f}  "
          f"bptt {bptt:.3f}  steps {len(fwd)}/{len(nb)}")
