#!/bin/bash
# A/B: -m local class words from the fused parse (build) against HEAD before
# them (build_b), C2 device path interleaved; then the GPU suite and the C2
# bench line on the new build (each step time-limited, first failure ends it)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
REPS=3 BUILDS="build build_b" timeout -k 10 600 bash tools/ab_builds.sh || { echo ab failed; exit 1; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo tests failed; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python3 -u bench.py --no-cpu > $O/bench_c2.json 2> $O/bench_c2.err || { echo bench failed; tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c2.json')); print('C2', d['value'], d['ms_per_step'], d['device_path']['ms_per_step'], d['device_path']['stages_ms'], d['roofline']['frac'])"
