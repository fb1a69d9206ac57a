#!/bin/bash
# round-3 re-entry check at HEAD: smoke, the whole GPU suite (bench-path
# parity included), the C2 and C3 bench lines, and the --gpus 2 rehearsal on
# one GPU (each step time-limited; the first failure ends the script)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo tests failed; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python3 -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo bench failed; tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c2.json')); print('C2', d['value'], d['ms_per_step'], d['device_path']['ms_per_step'], d['device_path']['stages_ms'], d['roofline']['frac'], d['roofline']['kernel'])"
timeout -k 10 400 python3 -u bench.py --config C3 --no-cpu > $O/bench_c3.json 2> $O/bench_c3.err || { echo c3 failed; tail $O/bench_c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c3.json')); print('C3', d['value'], d['ms_per_step'], d['device_path']['ms_per_step'], d['device_path']['stages_ms'])"
timeout -k 10 400 python3 -u bench.py --gpus 2 --allow-shared-gpu --no-cpu > $O/bench_2r.json 2> $O/bench_2r.err || { echo 2r failed; tail $O/bench_2r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_2r.json')); print('2r', d['value'], d['n_gpus'], d['config']['ranks'], d['config']['oversubscribed'], d['config']['rccl_world'])"
