"""Summarise a rocprofv3 --stats kernel_stats.csv: per-kernel total / calls / average."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:n]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f}ms {float(r['Percentage']):6.2f}% n={r['Calls']:>5} "
          f"avg={float(r['AverageNs'])/1e3:9.1f}us {r['Name'][:100]}")
print(f"total {tot/1e6:.2f} ms")
