#!/bin/bash
# round-2 state check on one GPU: smoke, GPU parity tests, C2 bench with extras,
# kernel trace of C2 (each step time-limited, first failure ends the call)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1 || { echo tests failed; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 400 python3 -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo bench failed; tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c2.json')); print(d['value'], d['ms_per_step'], d['stages_ms'], d['roofline'])"
bash tools/gpu_trace_c2.sh
