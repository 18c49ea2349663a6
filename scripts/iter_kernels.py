"""Kernels of one training iteration from a rocprofv3 kernel_trace.csv.

Iterations are split at the weight repack (``pack_gather_kernel``, the last launch of a step; it
runs the optimizer's commit since round 6). Prints, for the last complete iteration: per-kernel-name launch counts and total device
time, the glue kernels (anything not in the ``mb::`` namespace, e.g. ``at::native`` fills / copies)
and the sum of the gaps between consecutive kernels on the compute queue.

    python scripts/iter_kernels.py gpurun_out/TAG/kernel_trace.csv [--iter -1] [--json out.json]
"""
import argparse
import csv
import json
from collections import OrderedDict


def iterations(path, marker="pack_gather_kernel"):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    its, cur = [], []
    for r in rows:
        cur.append(r)
        if marker in r["Kernel_Name"]:
            its.append(cur)
            cur = []
    return its


def summary(it):
    names = OrderedDict()
    for r in it:
        n = r["Kernel_Name"]
        d = names.setdefault(n, [0, 0.0])
        d[0] += 1
        d[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    glue = {n: v for n, v in names.items() if not (n.startswith("mb::") or "mb::" in n.split("(")[0])}
    t0 = int(it[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in it)
    busy_end, idle = t0, 0
    for r in it:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s > busy_end:
            idle += s - busy_end
        busy_end = max(busy_end, e)
    return {"kernels": sum(v[0] for v in names.values()), "span_us": (t1 - t0) / 1e3, "idle_us": idle / 1e3,
            "by_name": {n: {"calls": v[0], "us": round(v[1], 1)} for n, v in names.items()},
            "glue": {n: v[0] for n, v in glue.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--iter", type=int, default=-1)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    its = iterations(a.trace)
    s = summary(its[a.iter])
    print(f"{len(its)} iterations; iteration {a.iter}: {s['kernels']} kernels, span {s['span_us']:.0f} us, "
          f"idle gaps {s['idle_us']:.0f} us")
    for n, v in sorted(s["by_name"].items(), key=lambda kv: -kv[1]["us"]):
        print(f"  {v['calls']:4d} x {v['us']:9.1f} us  {n[:110]}")
    print("glue (non-mb) kernels:", s["glue"] or "none")
    if a.json:
        json.dump(s, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
