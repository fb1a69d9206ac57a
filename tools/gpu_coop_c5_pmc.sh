#!/bin/bash
# the cooperative parse on the C5 shard (200x): stall split and instruction
# mix of its kernels (SID_PARSE_COOP=1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
export SID_PARSE_COOP=1
B="python3 $GRAFT_REPO_ROOT/bench.py --config C5 --sites 12500000 --steps 1"
run() {
    local g=$1; shift
    ( cd /tmp && timeout -s KILL 200 rocprofv3 --pmc "$@" --output-format csv -d $O/c5coop/pmc_$g -o p -- $B > $O/c5coop_$g.log 2>&1 )
}
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS || exit $?
run sq2 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS_ATOMIC SQ_BUSY_CYCLES || exit $?
( cd /tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5coop/trace -o t -- $B > $O/c5coop_trace.log 2>&1 ) || exit $?
echo done
