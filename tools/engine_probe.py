#!/usr/bin/env python3
"""Probe of the streaming engine at C2 size (50M 30x sites by default):

  device   text resident in HBM -> index, parse, call, format -> CSV records
           left in HBM (device sink): the whole text -> CSV path on the GPU
  host     the same text in host memory (pageable or pinned) -> H2D -> ... ->
           CSV D2H into host memory (PCIe both ways)

Prints one JSON line per configuration.  Usage:
  python tools/engine_probe.py [--sites N] [--runs K] [--chunk-mib M] [--modes device,host,pinned]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sites", type=int, default=50_000_000)
    ap.add_argument("--depth", type=float, default=30.0)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--chunk-mib", type=int, default=0)
    ap.add_argument("--method", default="local")
    ap.add_argument("--modes", default="device,host")
    a = ap.parse_args()
    import torch
    import sid_amd
    n = a.sites
    ctx = sid_amd.Context(0)
    cap = int(n * (30 + 3.0 * a.depth)) + (64 << 20)
    buf = torch.empty(cap + 512, dtype=torch.uint8, device="cuda")
    t0 = time.perf_counter()
    ln = ctx.synth_text_device(a.seed, a.depth, 0, n, buf.data_ptr(), cap)
    buf[ln:ln + 512].zero_()
    torch.cuda.synchronize()
    print(json.dumps({"generated_bytes": ln, "gen_s": time.perf_counter() - t0}), flush=True)
    kw = dict(method=a.method, chunk_bytes=a.chunk_mib << 20, estimate_prior=a.method != "local")
    for mode in a.modes.split(","):
        if mode == "device":
            eng = sid_amd.Engine(device_sink=True, **kw)
            eng.source_device_text(buf.data_ptr(), ln, keep=buf)
            sink = None
        else:
            host = buf[:ln].cpu()
            if mode == "pinned":
                host = host.pin_memory()
            eng = sid_amd.Engine(**kw)
            eng.source_host_ptr(host.data_ptr(), ln, keep=host)
            sink = os.open(os.devnull, os.O_WRONLY)
        runs = []
        for r in range(a.runs + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st = eng.ingest()
            eng.estimate()
            if sink is None:
                _, st2 = eng.emit()
            else:
                _, st2 = eng.emit(sink=sink)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            if r:
                runs.append({"s": dt, "ingest_s": st.ingest_s, "emit_s": st2.emit_s})
        best = min(runs, key=lambda x: x["s"])
        print(json.dumps({"mode": mode, "sites": st.sites, "chunks": st.chunks, "held": st.chunks_held,
                          "bytes_in": ln, "bytes_out": st2.bytes_out, "best_s": best["s"],
                          "sites_per_s": st.sites / best["s"], "runs": runs}), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
