#!/bin/bash
# quick perf iteration: C2 bench (no extras) + kernel trace summary, no tests
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u bench.py --no-extras "$@" > $O/bench_perf.json 2> $O/bench_perf.err || { tail -5 $O/bench_perf.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/bench_perf.json"))
print(f"value={d['value']:.4g} ms/step={d['ms_per_step']:.3f}", {k: round(v, 3) for k, v in d["stages_ms"].items()})
PY
bash tools/gpu_trace_c2.sh "$@"
