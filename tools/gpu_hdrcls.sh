#!/bin/bash
# class words in the header words (build) against HEAD (build_c: the 4 B
# class-word array) and before class words (build_b): C2 device path A/B;
# the GPU suite; PMC fetch/write passes of the device path; the C2 bench line
# (each step time-limited, the first failure ends it)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O/r03pmc3
export TMPDIR=/tmp
REPS=3 BUILDS="build build_c build_b" timeout -k 10 600 bash tools/ab_builds.sh || { echo ab failed; exit 1; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo tests failed; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
B="python3 $GRAFT_REPO_ROOT/bench.py --device-only --steps 2 --device-steps 2"
run() {
    local g=$1; shift
    ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/r03pmc3/pmc_$g -o p -- $B > $O/r03pmc3_$g.log 2>&1 )
}
run insts SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit $?
run fetch FETCH_SIZE || exit $?
run write WRITE_SIZE || exit $?
timeout -k 10 200 $B > $O/r03pmc3/pmc_bench.json 2>/dev/null || exit $?
python3 tools/pmc_summary.py $O/r03pmc3 --json $O/r03pmc3/summary.json > $O/r03pmc3/summary.txt || exit $?
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03trace -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu > $O/r03trace.json 2> $O/r03trace.log ) || { echo trace failed; tail $O/r03trace.log; exit 1; }
timeout -k 10 400 python3 -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo bench failed; tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c2.json')); print('C2', d['value'], d['ms_per_step'], d['device_path']['ms_per_step'], d['device_path']['stages_ms'], d['roofline']['frac'])"
