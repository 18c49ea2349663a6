"""Summarise rocprofv3 --pmc csv passes: per kernel, per-dispatch averages of every counter."""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.defaultdict(collections.Counter)
for path in sys.argv[1:]:
    for x in csv.DictReader(open(path)):
        k = x["Kernel_Name"].split("(")[0].replace("void ", "")[:44]
        agg[k][x["Counter_Name"]] += float(x["Counter_Value"])
        calls[k][x["Counter_Name"]] += 1
for k in sorted(agg, key=lambda k: -agg[k].get("SQ_WAVE_CYCLES", 0)):
    v = agg[k]
    row = {c: v[c] / calls[k][c] for c in v}
    if row.get("SQ_WAVE_CYCLES", 0) < 1e5 and row.get("SQ_BUSY_CYCLES", 0) < 1e5:
        continue
    print(k)
    print("   " + "  ".join(f"{c.replace('SQ_', '')}={val:.3g}" for c, val in sorted(row.items())))
