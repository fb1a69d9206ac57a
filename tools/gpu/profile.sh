#!/bin/bash
# rocprofv3 evidence for one config (MI355X_MICROARCH.md: TMPDIR=/tmp, the
# counters in passes of their own, never with the trace domains):
#   trace   --kernel-trace --stats over the bench as the driver runs it
#   dtrace  the same over the device path only (--device-only)
#   insts / fetch / write / stall / lds   --pmc passes over the device path
# then tools/pmc_summary.py -> gpurun_out/prof_<TAG>/summary.json and, with
# STAGES=1, tools/pmc_stages.py -> profiles/pmc_<stage>_<TAG>.json
# usage: PASSES="trace dtrace insts fetch write" tools/gpu/profile.sh TAG [--config C2]
. "$(dirname "$0")/common.sh"
TAG=${1:-run}; shift
P=$O/prof_$TAG
mkdir -p $P
B="python3 $PWD/bench.py --device-only --steps 2 --device-steps 2 $*"
pmc() {   # group counters...
    local g=$1; shift
    ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $P/pmc_$g -o p -- $B > $P/pmc_$g.log 2>&1 ) \
        || { echo "pmc $g failed"; tail -3 $P/pmc_$g.log; exit 1; }
}
for pass in ${PASSES:-trace dtrace insts fetch write}; do
    case $pass in
    trace) ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o trace -- \
               python3 $OLDPWD/bench.py --steps 20 --warmup 5 --no-cpu "$@" > $P/trace.json 2> $P/trace.log ) \
               || { echo "trace failed"; tail -3 $P/trace.log; exit 1; } ;;
    dtrace) ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/dtrace -o trace -- \
               python3 $OLDPWD/bench.py --device-only --steps 10 "$@" > $P/dtrace.json 2> $P/dtrace.log ) \
               || { echo "dtrace failed"; tail -3 $P/dtrace.log; exit 1; } ;;
    insts) pmc insts SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES ;;
    fetch) pmc fetch FETCH_SIZE ;;
    write) pmc write WRITE_SIZE ;;
    lds) pmc lds SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVES ;;
    stall) pmc stall SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS ;;
    esac
    echo "$pass ok"
done
for t in trace dtrace; do
    [ -f $P/$t/trace_kernel_stats.csv ] && python3 - $P/$t/trace_kernel_stats.csv <<'PY'
import csv, sys
print(sys.argv[1].split("/")[-2])
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:80]}")
PY
done
if ls $P/pmc_* > /dev/null 2>&1; then
    timeout -k 10 200 $B > $P/pmc_bench.json 2>/dev/null || { echo "pmc bench failed"; exit 1; }
    python3 tools/pmc_summary.py $P --json $P/summary.json > $P/summary.txt && head -12 $P/summary.txt
    [ -n "$STAGES" ] && python3 tools/pmc_stages.py $P $P/pmc_bench.json $TAG
fi
true
