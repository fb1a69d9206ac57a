#!/bin/bash
# device-path stage check, then the round-3 evidence: rocprofv3 kernel trace
# (--stats) of the C2 bench as the driver runs it, the PMC passes of the
# device path, the C3 line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo bench failed; tail $O/bench_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c2.json')); print('C2', d['value'], d['ms_per_step'], d['pcie']['ceiling']['frac'], d['device_path']['ms_per_step'], {k: round(v,3) for k,v in d['device_path']['stages_ms'].items()}, d['roofline']['frac'], d['cpu_baseline']['value'])"
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03trace -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu > $O/r03trace.json 2> $O/r03trace.log ) || { echo trace failed; tail $O/r03trace.log; exit 1; }
python3 - <<'PY'
import csv, os
p = os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out/r03trace/trace_kernel_stats.csv")
for r in list(csv.DictReader(open(p)))[:14]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:80]}")
PY
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
head -40 $O/r03pmc/summary.txt
timeout -k 10 400 python3 -u bench.py --config C3 --no-cpu > $O/bench_c3.json 2> $O/bench_c3.err || { echo c3 failed; tail $O/bench_c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c3.json')); print('C3', d['value'], d['ms_per_step'], d['device_path']['ms_per_step'], {k: round(v,3) for k,v in d['device_path']['stages_ms'].items()}, d['estimate'])"
