#!/bin/bash
# round 3: the whole GPU suite but the full-size bench-path tests, smoke, the
# C2 bench, the --gpus 2 rehearsal (each step time-limited, first failure ends)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --ignore tests/test_benchpath_gpu.py ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1 || { echo tests failed; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python3 -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo bench failed; tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c2.json')); print(d['value'], d['ms_per_step'], d['device_path']['ms_per_step'], d['device_path']['stages_ms'], d['roofline']['frac'])"
timeout -k 10 400 python3 -u bench.py --gpus 2 --allow-shared-gpu --steps 5 --warmup 2 --no-extras > $O/bench_2r.json 2> $O/bench_2r.err || { echo 2r failed; tail -20 $O/bench_2r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_2r.json')); print(d['value'], d['n_gpus'], d['config']['ranks'], d['config']['oversubscribed'])"
