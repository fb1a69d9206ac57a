#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc passes of tools/gpu/profile.sh: per kernel, the
average per launch of every counter collected, HBM bytes per launch
(FETCH_SIZE x 1024 x 2 -- gfx950 reports half the bytes of wide coalesced
reads, MI355X_MICROARCH.md §HBM -- + WRITE_SIZE x 1024) and the wave
instruction mix.  usage: tools/pmc_summary.py <dir with pmc_* subdirs> [--json out.json]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    n = name
    for pre in ("(anonymous namespace)::", "void "):
        n = n.replace(pre, "")
    return n.split("(")[0].split("<")[0]


def main():
    src = sys.argv[1]
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(src, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in sorted(vals.items()):
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        launches = max(len(v) for v in cs.values())
        row = {"launches": launches, **{c: round(a, 1) for c, a in avg.items()}}
        if "FETCH_SIZE" in avg or "WRITE_SIZE" in avg:
            row["hbm_bytes"] = avg.get("FETCH_SIZE", 0.0) * 1024 * 2 + avg.get("WRITE_SIZE", 0.0) * 1024
        out[k] = row
    for k, r in sorted(out.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", kv[1].get("hbm_bytes", 0))):
        print(k, json.dumps(r))
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
