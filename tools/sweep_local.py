#!/usr/bin/env python3
"""A/B sweep of the -m local kernel variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  Variants are selected through the
SID_* environment knobs read at context creation.  Prints one JSON line per
variant: median / min kernel ms over rounds and the algorithmic GB/s."""
import itertools
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import sid_amd
    n = int(os.environ.get("SWEEP_SITES", 50_000_000))
    depth = float(os.environ.get("SWEEP_DEPTH", 30.0))
    rounds = int(os.environ.get("SWEEP_ROUNDS", 5))
    reps = int(os.environ.get("SWEEP_REPS", 5))
    dev = torch.device("cuda", 0)
    counts = torch.empty((n, 4), dtype=torch.int16, device=dev)
    code = torch.empty(n, dtype=torch.uint8, device=dev)
    hom = torch.empty(n, dtype=torch.float64, device=dev)
    het = torch.empty(n, dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev)
    variants = [dict(SID_LOCAL_DIRECT="1")]
    grids = os.environ.get("SWEEP_GRIDS", "512,1024,2048,4096,8192").split(",")
    unrolls = os.environ.get("SWEEP_UNROLLS", "1,2").split(",")
    for u, nt, g, ch in itertools.product(unrolls, ["0", "1"], grids, ["0", "1"]):
        variants.append(dict(SID_TABLE_UNROLL=u, SID_TABLE_NT=nt, SID_TABLE_GRID=g, SID_TABLE_CHUNK=ch))
    ctxs = []
    for v in variants:
        for k in ("SID_LOCAL_DIRECT", "SID_TABLE_UNROLL", "SID_TABLE_NT", "SID_TABLE_GRID", "SID_TABLE_CHUNK"):
            os.environ.pop(k, None)
        os.environ.update(v)
        ctxs.append(sid_amd.Context(0))
    ctxs[0].synth_counts(2, depth, 0, n, counts.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    times = [[] for _ in variants]
    ref = None
    for r in range(rounds):
        for i, c in enumerate(ctxs):
            c.call_local(counts.data_ptr(), n, code.data_ptr(), hom.data_ptr(), het.data_ptr(), st.cuda_stream)
            torch.cuda.synchronize()
            if r == 0:   # every variant must produce the same bytes
                sig = (int(code.sum().item()), float(hom.sum().item()), float(het.sum().item()))
                ref = ref or sig
                assert sig == ref, (variants[i], sig, ref)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(st)
            for _ in range(reps):
                c.call_local(counts.data_ptr(), n, code.data_ptr(), hom.data_ptr(), het.data_ptr(), st.cuda_stream)
            e.record(st)
            torch.cuda.synchronize()
            times[i].append(s.elapsed_time(e) / reps)
    for v, t in zip(variants, times):
        t = sorted(t)
        med = t[len(t) // 2]
        print(json.dumps({"variant": v, "median_ms": med, "min_ms": t[0],
                          "GBps_median": 25 * n / (med * 1e-3) / 1e9, "sites": n, "depth": depth}), flush=True)


if __name__ == "__main__":
    main()
