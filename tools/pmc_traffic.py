#!/usr/bin/env python3
"""Turn the rocprofv3 outputs of tools/profile_round.sh into the committed
summaries under profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_pmc.csv            per-kernel FETCH_SIZE / WRITE_SIZE averages
  profiles/<tag>_summary.json       per-kernel average duration, HBM bytes per
                                    launch (FETCH_SIZE x 1024 x 2 -- gfx950
                                    reports half the bytes of a wide
                                    coalesced read, MI355X_MICROARCH.md §HBM --
                                    + WRITE_SIZE x 1024), algorithmic bytes
  profiles/pmc_<tag>.json           what bench.py reads for roofline.traffic
                                    (the first kernel named below)

usage: tools/pmc_traffic.py <gpurun_out dir> <prefix> <tag> <sites> KERNEL:BYTES_PER_SITE [...]
  prefix: the PREFIX given to profile_round.sh (dirs <prefix>_trace, _fetch, _write)
  e.g.    tools/pmc_traffic.py gpurun_out local local_r01 50000000 sid_local_table_p2:25
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    n = name
    for pre in ("(anonymous namespace)::", "void "):
        n = n.replace(pre, "")
    return n.split("(")[0]


def main():
    src, prefix, tag, sites = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    algo = [(k.split(":")[0], float(k.split(":")[1])) for k in sys.argv[5:]]
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = os.path.join(src, f"{prefix}_trace", "trace_kernel_stats.csv")
    shutil.copy(stats, os.path.join(out, f"{tag}_kernel_stats.csv"))
    dur = {}
    for r in csv.DictReader(open(stats)):
        dur[short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]))
    pmc = defaultdict(list)
    for sub, fn in (("fetch", "fetch_counter_collection.csv"), ("write", "write_counter_collection.csv")):
        p = os.path.join(src, f"{prefix}_{sub}", fn)
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            pmc[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    if pmc:
        with open(os.path.join(out, f"{tag}_pmc.csv"), "w") as f:
            f.write("kernel,counter,launches,average_kb\n")
            for (k, c), v in sorted(pmc.items()):
                f.write(f"{k},{c},{len(v)},{sum(v) / len(v):.3f}\n")
    summary = {"sites_per_launch": sites, "kernels": {}}
    for k, (calls, ns) in dur.items():
        fetch = pmc.get((k, "FETCH_SIZE"))
        write = pmc.get((k, "WRITE_SIZE"))
        e = {"calls": calls, "avg_ns": ns}
        if fetch:
            e["fetch_bytes_corrected"] = sum(fetch) / len(fetch) * 1024 * 2
        if write:
            e["write_bytes"] = sum(write) / len(write) * 1024
        if fetch and write:
            e["hbm_bytes_per_launch"] = e["fetch_bytes_corrected"] + e["write_bytes"]
        summary["kernels"][k] = e
    first = True
    for kname, bps in algo:
        hits = [k for k in summary["kernels"] if k.startswith(kname)]
        if not hits:
            continue
        e = summary["kernels"][hits[0]]
        alg = bps * sites
        if alg <= 0:
            continue
        e["algorithmic_bytes"] = alg
        e["achieved_GBps"] = alg / e["avg_ns"]
        if "hbm_bytes_per_launch" in e:
            e["traffic_over_algorithmic"] = e["hbm_bytes_per_launch"] / alg
            if first:
                json.dump({"sites": sites, "kernel": hits[0], "hbm_bytes_per_launch": e["hbm_bytes_per_launch"],
                           "source": f"profiles/{tag}_pmc.csv (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE)"},
                          open(os.path.join(out, f"pmc_{tag}.json"), "w"), indent=1)
        first = False
    json.dump(summary, open(os.path.join(out, f"{tag}_summary.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
