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
P=${PREFIX:-prof}
PASSES=${PASSES:-"trace fetch write"}
case " $PASSES " in *" trace "*)
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${P}_trace -o trace -- \
    python3 bench.py $ARGS > $O/${P}_trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo "trace ok" ;; esac
case " $PASSES " in *" fetch "*)
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${P}_fetch -o fetch -- \
    python3 bench.py $ARGS > $O/${P}_fetch.log 2>&1 || { echo "fetch rc=$?"; exit 1; }
echo "fetch ok" ;; esac
case " $PASSES " in *" write "*)
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${P}_write -o write -- \
    python3 bench.py $ARGS > $O/${P}_write.log 2>&1 || { echo "write rc=$?"; exit 1; }
echo "write ok" ;; esac
