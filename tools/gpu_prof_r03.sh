#!/bin/bash
# kernel trace + PMC passes of the C2 device path (bench.py --device-only):
# per-kernel time, instruction mix / stall counters, HBM bytes (FETCH_SIZE and
# WRITE_SIZE in their own passes, MI355X_MICROARCH.md).  Output gpurun_out/prof_*
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --device-only --steps 4 --device-steps 4 ${BENCH_ARGS}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_trace -o trace -- $B > $O/prof_trace.log 2>&1 || exit $?
python3 - <<'PY'
import csv, os
p = os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out/prof_trace/trace_kernel_stats.csv")
for r in list(csv.DictReader(open(p)))[:16]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:90]}")
PY
run() {   # group counters...
    local g=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/pmc_$g -o p -- $B > $O/pmc_$g.log 2>&1
}
run insts SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit $?
run stall SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU SQ_WAVE_CYCLES || echo "stall pass failed: $?"
run fetch FETCH_SIZE || exit $?
run write WRITE_SIZE || exit $?
timeout -k 10 200 $B > $O/pmc_bench.json 2>/dev/null || exit $?
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $O
