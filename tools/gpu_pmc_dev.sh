#!/bin/bash
# PMC passes of the C2 device path (2 GiB chunks, 25M-site launches), one
# counter group per rocprofv3 run (MI355X_MICROARCH.md), then the summary for
# tools/pmc_stages.py; and the C3 bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O/r03pmc
export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --device-only --steps 2 --device-steps 2"
run() {
    local g=$1; shift
    ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/r03pmc/pmc_$g -o p -- $B > $O/r03pmc_$g.log 2>&1 )
}
run insts SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit $?
run fetch FETCH_SIZE || exit $?
run write WRITE_SIZE || exit $?
timeout -k 10 200 $B > $O/r03pmc/pmc_bench.json 2>/dev/null || exit $?
python3 tools/pmc_summary.py $O/r03pmc --json $O/r03pmc/summary.json > $O/r03pmc/summary.txt || exit $?
timeout -k 10 400 python3 -u bench.py --config C3 --no-cpu > $O/bench_c3.json 2> $O/bench_c3.err || { echo c3 failed; tail $O/bench_c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c3.json')); print('C3', d['value'], d['ms_per_step'], d['device_path']['ms_per_step'], {k: round(v,3) for k,v in d['device_path']['stages_ms'].items()})"
