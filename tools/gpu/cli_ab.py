#!/usr/bin/env python3
"""A/B of CLI builds on one box: the C2 text (50M sites, seed 2) as a file in
the page cache, then each binary `--stats FILE > /dev/null` in turn, REPS
rounds; wall clock around the process and the CLI's own clock, one JSON line
per run, then the median wall per binary.

usage: python3 tools/gpu/cli_ab.py OUT.jsonl build/sid build_dev/sid [...]
env:   REPS (5), SITES (50000000), and per binary any KEY=VALUE given as
       BIN:KEY=VALUE (e.g. build/sid:SID_UPLOAD_REGISTER=0)
"""
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    out, bins = sys.argv[1], sys.argv[2:]
    import bench
    from sid_amd import gpu as G
    n = int(os.environ.get("SITES", 50_000_000))
    text, ln = G.synth_text_hbm(2, 30.0, 0, n, device=0)
    runs = {b: [] for b in bins}
    with tempfile.TemporaryDirectory() as td, open(out, "w") as fo:
        path = os.path.join(td, "c2.plp")
        bench.write_text_file(text, ln, path)
        del text
        for r in range(int(os.environ.get("REPS", 5)) + 1):
            for spec in bins:
                b, _, kv = spec.partition(":")
                env = dict(os.environ)
                if kv:
                    k, v = kv.split("=", 1)
                    env[k] = v
                with open(os.devnull, "wb") as dn:
                    u0 = time.time()
                    t0 = time.perf_counter()
                    p = subprocess.run([os.path.join(ROOT, b), "--stats", path], stdout=dn, stderr=subprocess.PIPE,
                                       env=env, timeout=120)
                    dt = time.perf_counter() - t0
                    u1 = time.time()
                if p.returncode != 0:
                    print(spec, "failed", p.returncode, p.stderr.decode()[-300:])
                    sys.exit(1)
                lines = p.stderr.decode().strip().splitlines()
                st = json.loads(lines[-1])
                # SID_ENGINE_TIMING=1: the engine's phase lines before it
                eng = [json.loads(x) for x in lines[:-1] if x.startswith('{"engine_phase"')]
                rec = {"bin": spec, "round": r, "wall_s": dt, "create_s": st.get("create_s"),
                       "total_s": st.get("total_s"), "emit_s": st.get("emit_s"), "parse_s": st.get("parse_s"),
                       "main_s": st["main_exit_unix"] - st["main_entry_unix"],
                       # process start to main, main's end to the parent's wait
                       "pre_s": st["main_entry_unix"] - u0, "post_s": u1 - st["main_exit_unix"],
                       "unmap_s": st.get("unmap_s"), "destroy_s": st.get("destroy_s"),
                       "chunks": st.get("chunks"),
                       "chunks_registered": sum(x.get("chunks_registered", 0) for x in eng) if eng else None}
                fo.write(json.dumps(rec) + "\n")
                fo.flush()
                if r:   # the first round warms the page cache and the code objects
                    runs[spec].append(dt)
    for spec, v in runs.items():
        print(f"{spec}: median wall {statistics.median(v):.3f} s  runs {[round(x, 3) for x in v]}")


if __name__ == "__main__":
    main()
