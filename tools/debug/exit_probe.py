#!/usr/bin/env python3
"""Runs build/exit_probe in each mode REPS times, interleaved; one JSON line a
run with post_s = the parent's wait returning minus the probe's last clock
reading (how long the process took to go away), then the median per mode.

usage: python3 tools/debug/exit_probe.py OUT.jsonl [REPS]
"""
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
MODES = ["init", "streams", "hbm", "pinned", "engine"]


def main():
    out = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    post = {m: [] for m in MODES}
    with open(out, "w") as fo:
        for r in range(reps):
            for m in MODES:
                p = subprocess.run([os.path.join(ROOT, "build", "exit_probe"), m], capture_output=True, timeout=60)
                u1 = time.time()
                if p.returncode != 0:
                    print(m, "failed", p.returncode, p.stderr.decode()[-300:])
                    sys.exit(1)
                st = json.loads(p.stdout.decode().strip().splitlines()[-1])
                rec = {"mode": m, "round": r, "rc": st["rc"], "post_s": u1 - st["main_exit_unix"]}
                fo.write(json.dumps(rec) + "\n")
                fo.flush()
                post[m].append(rec["post_s"])
    for m, v in post.items():
        print(f"{m}: median post {statistics.median(v) * 1e3:.1f} ms  runs {[round(x * 1e3, 1) for x in v]}")


if __name__ == "__main__":
    main()
