"""Run the cooperative-parse stress texts (tests/test_parse_stress_gpu.py)
through the CLIs of two builds and the oracle CLI, each call under a time
limit, printing one line per call (which case is slow or differs)."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import sid_amd as sid  # noqa: E402
import oracle as O  # noqa: E402
from test_parse_stress_gpu import stress_text  # noqa: E402

out = os.path.join(ROOT, "gpurun_out")
os.makedirs(out, exist_ok=True)
builds = sys.argv[1:] or ["build"]
for seed, depth, n in [(41, 30.0, 20000), (43, 200.0, 6000)]:
    p = os.path.join("/tmp", f"stress_{seed}.plp")
    open(p, "wb").write(stress_text(sid, seed, n, depth))
    ref = O.run_cli([p])
    refR = O.run_cli(["-R", "-m", "likelihood_ratio", p])
    for b in builds:
        for extra in (["--chunk-bytes", "300000", "-R", "-m", "likelihood_ratio"],
                      ["--chunk-bytes", str(1 << 20), "-R", "-m", "likelihood_ratio"],
                      ["--chunk-bytes", str(1 << 20)], ["--chunk-bytes", "65537", "--devices", "2"],
                      ["--chunk-bytes", "20000"]):
            t = time.time()
            try:
                r = subprocess.run([os.path.join(ROOT, b, "sid")] + extra + [p], capture_output=True, timeout=60)
                want = refR if "-R" in extra else ref
                res = (r.returncode, r.stdout == want.stdout, r.stderr == want.stderr, r.stderr[-200:])
            except subprocess.TimeoutExpired:
                res = ("TIMEOUT",)
            print(seed, b, extra, f"{time.time() - t:.2f}s", res, flush=True)
