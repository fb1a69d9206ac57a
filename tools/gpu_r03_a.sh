#!/bin/bash
# round 3, first GPU call: the new engine tests (host arena), the full-size
# bench-path parity tests, the PCIe-inclusive C2 bench, and the --gpus 2
# rehearsal (ranks spawned by bench.py itself) + its refusal without the flag
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_engine_gpu.py -k "host or exchange or past_eof" > $O/pytest_hh.log 2>&1 || { echo hh tests failed; tail -40 $O/pytest_hh.log; exit 1; }
tail -2 $O/pytest_hh.log
timeout -k 10 400 python3 -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo bench failed; tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c2.json')); print(d['value'], d['ms_per_step'], d['pcie'], d['device_path']['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_2r.json 2> $O/bench_2r.err && { echo "2 ranks on 1 GPU NOT refused"; exit 1; }
tail -1 $O/bench_2r.err
timeout -k 10 400 python3 -u bench.py --gpus 2 --allow-shared-gpu --steps 5 --warmup 2 > $O/bench_2r.json 2> $O/bench_2r.err || { echo 2r failed; tail -20 $O/bench_2r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_2r.json')); print(d['value'], d['n_gpus'], d['config']['ranks'], d['config']['oversubscribed'])"
timeout -k 10 800 $T --timeout 780 tests/test_benchpath_gpu.py > $O/pytest_benchpath.log 2>&1 || { echo benchpath tests failed; tail -40 $O/pytest_benchpath.log; exit 1; }
tail -3 $O/pytest_benchpath.log
