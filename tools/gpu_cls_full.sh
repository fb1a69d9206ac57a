#!/bin/bash
# class words, final form: A/B against HEAD before them (build_b), the GPU
# suite, the PMC passes (tools/gpu_pmc_c2.sh), the C2 kernel trace and the
# C2 bench line (each step time-limited, the first failure ends it)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
export TMPDIR=/tmp
REPS=3 BUILDS="build build_b" timeout -k 10 600 bash tools/ab_builds.sh || { echo ab failed; exit 1; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo tests failed; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/gpu_pmc_c2.sh > $O/pmc_summary.txt 2>&1 || { echo pmc failed; tail $O/pmc_summary.txt; exit 1; }
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03trace -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu > $O/r03trace.json 2> $O/r03trace.log ) || { echo trace failed; tail $O/r03trace.log; exit 1; }
timeout -k 10 400 python3 -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo bench failed; tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c2.json')); print('C2', d['value'], d['ms_per_step'], d['device_path']['ms_per_step'], d['device_path']['stages_ms'], d['roofline']['frac'])"
