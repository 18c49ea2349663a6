"""Speed-of-light table of every kernel of the training iteration from ONE workload: the PMC
passes of scripts/gpu_sol.sh run bench.py itself (the headline iteration), and the durations are
the same dispatches' own timestamps in the counter-collection CSV -- counters and times never
mix workloads.

Per kernel (per-dispatch averages over the collected dispatches):
  us        end - start timestamp of the dispatch (counter collection serialises dispatches: this
            is the kernel alone; the bench's wall time also holds overlap and launch gaps)
  MFMA us   SQ_INSTS_MFMA x cycles per MFMA / (1024 SIMDs x 2.4 GHz); 16 cycles for the
            v_mfma_f32_16x16x32_bf16 kernels (names containing 16_kernel), else 32
            (v_mfma_f32_32x32x16_bf16) -- MI355X_MICROARCH.md cycle constants
  VALU us   SQ_INSTS_VALU x 2 cycles / (1024 x 2.4 GHz): a wave64 VALU instruction occupies its
            SIMD-32 for 2 cycles (4 is the issue cost of ONE wave's stream; with two or more waves
            per SIMD the SIMD's rate is the bound)
  issue us  max(MFMA cycles, VALU x 2 + MFMA x 8) / (1024 x 2.4 GHz): an MFMA blocks its SIMD's
            vector issue for 8 of its cycles (MI355X_MICROARCH.md constants table)
  The clock is the nominal 2.4 GHz: under this load the shader clock runs lower (s_memtime phase
  clocks vs wall time: ~1.8-2.1 GHz), so the SOL column understates the utilisation by that ratio.
  SOL %     issue us / us
  conflicts SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  active    SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES

    python scripts/sol_table.py OUT.md PASS1/counter_collection.csv PASS2/counter_collection.csv ...
"""
import csv
import json
import sys
from collections import defaultdict

CLK = 2.4e9
SIMDS = 1024


def short(name: str) -> str:
    n = name.split("(")[0]
    for p in ("void ", "mb::x3::", "mb::f16::", "mb::"):
        n = n.replace(p, "")
    return n


def load(paths):
    # keyed by (pass, kernel, dispatch): the passes are separate runs of one deterministic program,
    # so their dispatch ids coincide -- a (kernel, dispatch) key would merge the passes' dispatches
    # and halve the dispatch count the per-dispatch averages divide by (the round-4 first table
    # reported every MFMA / VALU column 2x too high this way)
    per = defaultdict(lambda: defaultdict(float))   # (pass, kernel, dispatch) -> counters
    times = {}
    for i, p in enumerate(paths):
        for r in csv.DictReader(open(p)):
            did = r.get("Dispatch_Id") or r.get("Correlation_Id")
            per[(i, r["Kernel_Name"], did)][r["Counter_Name"]] += float(r["Counter_Value"])
            if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                times.setdefault((r["Kernel_Name"], did), {})[i] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    agg = defaultdict(lambda: defaultdict(float))
    for (_, kname, _), c in per.items():
        a = agg[kname]
        a["dispatches"] += 1
        for cn, v in c.items():
            a[cn] += v
    for (kname, did), ts in times.items():
        agg[kname]["ns_sum"] += sum(ts.values()) / len(ts)      # one duration per dispatch (passes averaged)
        agg[kname]["ns_n"] += 1
    return agg


def main():
    out, paths = sys.argv[1], sys.argv[2:]
    agg = load(paths)
    rows = []
    for k, a in agg.items():
        us = a["ns_sum"] / max(a["ns_n"], 1) / 1e3 if a["ns_n"] else float("nan")
        mf = a.get("SQ_INSTS_MFMA", 0.0)
        va = a.get("SQ_INSTS_VALU", 0.0)
        cyc_mfma = 16 if "16_kernel" in k else 32
        # each counter appears in exactly one pass: divide by the dispatches that pass saw
        d_each = a["dispatches"] / max(len(paths), 1)
        mf_d, va_d = mf / d_each, va / d_each
        mfma_us = mf_d * cyc_mfma / SIMDS / CLK * 1e6
        valu_us = va_d * 2 / SIMDS / CLK * 1e6
        issue_us = max(mf_d * cyc_mfma, va_d * 2 + mf_d * 8) / SIMDS / CLK * 1e6
        confl = a.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(a.get("SQ_LDS_IDX_ACTIVE", 0.0), 1.0)
        act = a.get("SQ_ACTIVE_INST_ANY", 0.0) / max(a.get("SQ_WAVE_CYCLES", 0.0), 1.0)
        tot_us = us * d_each
        rows.append(dict(kernel=short(k), dispatches=int(d_each), us=us, total_us=tot_us, mfma_us=mfma_us,
                         valu_us=valu_us, issue_us=issue_us, sol=issue_us / us if us == us and us > 0 else float("nan"),
                         conflicts=confl, active=act, mfma_per_disp=mf_d, valu_per_disp=va_d))
    rows.sort(key=lambda r: -r["total_us"])
    lines = ["| kernel | calls | us / call | MFMA us | VALU us | issue bound us | SOL % | LDS conflicts | wave cycles active |",
             "|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        if r["total_us"] < 1.0:
            continue
        lines.append(f"| {r['kernel']} | {r['dispatches']} | {r['us']:.1f} | {r['mfma_us']:.1f} | {r['valu_us']:.1f} | "
                     f"{r['issue_us']:.1f} | {100 * r['sol']:.0f} % | {100 * r['conflicts']:.0f} % | {100 * r['active']:.0f} % |")
    open(out, "w").write("\n".join(lines) + "\n")
    json.dump(rows, open(out.rsplit(".", 1)[0] + ".json", "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
