#!/usr/bin/env python3
"""Per-stage HBM traffic of the engine from the rocprofv3 --pmc passes of
tools/gpu/profile.sh, written as profiles/pmc_<stage>_<tag>.json for bench.py's
roofline.traffic (bytes per site x the sites of a launch).

Bytes per launch of a kernel: FETCH_SIZE x 1024 x 2 (gfx950 reports half the
bytes of a wide coalesced read, MI355X_MICROARCH.md §HBM) + WRITE_SIZE x 1024;
a stage's bytes = the sum over its kernels (bench.py STAGE_KERNELS).

usage: tools/pmc_stages.py <gpurun_out dir> <bench json of the same run> <tag>
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STAGES = {   # the scan kernels (shared by the index and the formatter, ~20 us) are left out
    "index": ["sid_index_count_kernel"],
    "parse": ["sid_index_emit_kernel", "sid_parse_kernel", "sid_parse_len_kernel", "sid_parse_quad_kernel",
              "sid_parse_serial_kernel", "sid_local_len_list_kernel",
              # the tile parse (-m local, lines up to 256 B): index, parse, lengths and fix-up in one stage
              "sid_tile_parse_kernel", "sid_tile_serial_kernel"],
    "call": ["sid_lookup_rec_kernel"],
    "hist": ["sid_hist_dense_kernel", "sid_hist_reduce_kernel", "sid_hist_list_kernel"],
    "fmt_len": ["sid_local_len_kernel", "sid_local_fixlen_kernel", "sid_fmt_blen_kernel", "sid_lynch_len_kernel"],
    "fmt_write": ["sid_local_put_kernel", "sid_fmt_put_kernel", "sid_lynch_put_kernel"],
}


def main():
    src, bench, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    tmp = os.path.join(src, "pmc_summary.json")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), src, "--json", tmp],
                   check=True, stdout=subprocess.DEVNULL)
    pm = json.load(open(tmp))
    b = json.load(open(bench))
    sites = b["roofline"]["sites_per_launch"]
    tile = "sid_tile_parse_kernel" in pm
    for stage, ks in STAGES.items():
        if tile and stage == "parse":
            # the tile parse's stage (the two-pass kernels only ran for chunks
            # whose tiles overflowed their slots: not the stage's steady state)
            ks = ["sid_tile_parse_kernel", "sid_tile_serial_kernel", "sid_tile_compact_kernel"]
        if tile and stage == "index":
            continue
        tot, parts = 0.0, {}
        for k in ks:
            r = pm.get(k)
            if not r or "hbm_bytes" not in r:
                continue
            parts[k] = r["hbm_bytes"]
            tot += parts[k]
        if not parts:
            continue
        out = {"stage": stage, "hbm_bytes_per_launch": tot, "sites_per_launch": sites,
               "hbm_bytes_per_site": tot / sites, "kernels": parts,
               "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes (tools/gpu/profile.sh); "
                         "FETCH_SIZE x 1024 x 2 + WRITE_SIZE x 1024 per launch, averaged over launches",
               "bench": os.path.basename(bench)}
        with open(os.path.join(ROOT, "profiles", f"pmc_{stage}_{tag}.json"), "w") as f:
            json.dump(out, f, indent=1)
        print(stage, round(tot / sites, 2), "B/site")


if __name__ == "__main__":
    main()
