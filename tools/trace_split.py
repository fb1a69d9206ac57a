#!/usr/bin/env python3
"""Per-kernel statistics of a rocprofv3 --kernel-trace CSV split by grid size,
so that the launches of one configuration (e.g. bench.py's device_path, 25M
sites per launch) are not averaged with another's (its 128 MiB PCIe-path
chunks).  usage: tools/trace_split.py trace_kernel_trace.csv [--top N] [--csv out]"""
import csv
import sys
from collections import defaultdict


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    g = defaultdict(list)
    for r in rows:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        g[(short(r["Kernel_Name"]), int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))].append(d)
    out = []
    for (k, grid, wg), ds in g.items():
        out.append({"kernel": k, "grid": grid, "workgroup": wg, "calls": len(ds), "total_ms": sum(ds) / 1e6,
                    "avg_us": sum(ds) / len(ds) / 1e3, "min_us": min(ds) / 1e3, "max_us": max(ds) / 1e3})
    out.sort(key=lambda r: -r["total_ms"])
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 25
    for r in out[:top]:
        print(f"{r['total_ms']:10.3f} ms {r['calls']:6d} x {r['avg_us']:9.1f} us (min {r['min_us']:8.1f})  "
              f"grid {r['grid']:>10} / {r['workgroup']:<5} {r['kernel']}")
    if "--csv" in sys.argv:
        with open(sys.argv[sys.argv.index("--csv") + 1], "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0]))
            w.writeheader()
            w.writerows(out)


if __name__ == "__main__":
    main()
