"""Per-kernel table from a prof_workload.py --summarize JSON (per-dispatch averages): waves,
cycles per wave, the wave-cycle split (active / waiting on counters / issue stalls), instruction
mix per wave and the LDS conflict share.

    python scripts/pmc_table.py gpurun_out/TAG/pmc.json
"""
import json
import sys


def main(path):
    d = json.load(open(path))
    print(f"{'kernel':58s} {'disp':>4s} {'waves':>6s} {'cyc/wave':>9s} {'active':>6s} {'wait':>5s} {'stall':>5s} "
          f"{'valu/w':>7s} {'mfma/w':>7s} {'lds/w':>6s} {'vmem/w':>6s} {'confl':>5s}")
    rows = sorted(d.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0) * kv[1].get("dispatches", 1))
    for k, r in rows:
        w = max(r.get("SQ_WAVES", 0), 1)
        cyc = r.get("SQ_WAVE_CYCLES", 0)
        f = lambda c: r.get(c, 0) / cyc if cyc else 0
        conf = r.get("SQ_LDS_BANK_CONFLICT", 0) / max(r.get("SQ_LDS_IDX_ACTIVE", 0), 1)
        print(f"{k[:58]:58s} {r.get('dispatches', 0):4d} {w:6.0f} {4 * cyc / w:9.0f} {f('SQ_ACTIVE_INST_ANY'):6.2f} "
              f"{f('SQ_WAIT_ANY'):5.2f} {f('SQ_WAIT_INST_ANY'):5.2f} {r.get('SQ_INSTS_VALU', 0) / w:7.0f} "
              f"{r.get('SQ_INSTS_MFMA', 0) / w:7.0f} {r.get('SQ_INSTS_LDS', 0) / w:6.0f} {r.get('SQ_INSTS_VMEM_RD', 0) / w:6.0f} "
              f"{conf:5.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
