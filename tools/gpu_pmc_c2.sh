#!/bin/bash
# PMC passes over a short C2 bench run (one counter group per rocprofv3 run, as
# MI355X_MICROARCH.md prescribes): instruction mix + HBM bytes per kernel.
# Output: gpurun_out/pmc_<group>/ ; summary printed by tools/pmc_summary.py
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
run() {   # group counters...
    local g=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/pmc_$g -o p -- \
        python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-extras > $O/pmc_$g.log 2>&1
}
run insts SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit $?
run fetch FETCH_SIZE || exit $?
run write WRITE_SIZE || exit $?
timeout -k 10 200 python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-extras > $O/pmc_bench.json 2>/dev/null || exit $?
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $O
