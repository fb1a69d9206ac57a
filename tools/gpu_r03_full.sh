#!/bin/bash
# round 3 state check: smoke, the whole GPU suite (full-size bench-path tests
# last), the C2 bench with every leg (each step time-limited, first failure ends)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --ignore tests/test_benchpath_gpu.py > $O/pytest_gpu.log 2>&1 || { echo tests failed; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python3 -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo bench failed; tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c2.json')); print(d['value'], d['ms_per_step'], d['device_path']['ms_per_step'], d['device_path']['stages_ms'], d['roofline']['frac'], d['roofline']['kernel'])"
timeout -k 10 900 python3 -u -m pytest tests/test_benchpath_gpu.py -m gpu -x -v --timeout 880 --timeout-method thread > $O/pytest_benchpath.log 2>&1 || { echo benchpath failed; grep -E "FAIL|Error|assert" $O/pytest_benchpath.log | head -20; tail -30 $O/pytest_benchpath.log; exit 1; }
tail -6 $O/pytest_benchpath.log
