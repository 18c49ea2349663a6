"""Per-iteration GPU busy / idle analysis of a rocprofv3 kernel trace (csv): splits the trace
into iterations at each scenario_kernel launch, merges the kernel intervals of all streams and
reports, per iteration, wall span, busy time (union of kernel intervals) and the largest idle gaps.

usage: python scripts/trace_gaps.py run_kernel_trace.csv [--marker scenario_kernel]
"""
import csv
import sys

path = sys.argv[1]
marker = sys.argv[3] if len(sys.argv) > 3 and sys.argv[2] == "--marker" else "scenario_kernel"
rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path))))
its, cur = [], []
for r in rows:
    if marker in r[2] and cur:
        its.append(cur)
        cur = []
    cur.append(r)
its.append(cur)
for k, it in enumerate(its):
    s0, e_max = it[0][0], max(r[1] for r in it)
    busy, gaps, end = 0, [], None
    for s, e, n in it:
        if end is None or s > end:
            if end is not None:
                gaps.append((s - end, n[:40]))
            busy += e - s
            end = e
        elif e > end:
            busy += e - end
            end = e
    gaps.sort(reverse=True)
    span = e_max - s0
    print(f"iter {k}: kernels {len(it)} span {span / 1e3:.1f} us busy {busy / 1e3:.1f} us idle {(span - busy) / 1e3:.1f} us "
          f"({len(gaps)} gaps); largest: " + ", ".join(f"{g / 1e3:.1f} before {n}" for g, n in gaps[:4]))
