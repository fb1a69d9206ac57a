#!/bin/bash
# rocprofv3 passes over a short bench run (TMPDIR=/tmp as the guide says):
#   1. --kernel-trace --stats        per-kernel durations
#   2. --pmc FETCH_SIZE              HBM read bytes   (separate pass)
#   3. --pmc WRITE_SIZE              HBM write bytes  (separate pass)
# Outputs under gpurun_out/prof_*; tools/pmc_traffic.py turns them into
# profiles/*.  Every step has its own time limit; the first failure ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
ARGS=${BENCH_ARGS:-"--steps 10 --warmup 2 --cpu-sample 0"}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_trace -o trace -- \
    python3 bench.py $ARGS > $O/prof_trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo "trace ok"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -o fetch -- \
    python3 bench.py $ARGS > $O/prof_fetch.log 2>&1 || { echo "fetch rc=$?"; exit 1; }
echo "fetch ok"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -o write -- \
    python3 bench.py $ARGS > $O/prof_write.log 2>&1 || { echo "write rc=$?"; exit 1; }
echo "write ok"
