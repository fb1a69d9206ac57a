#!/bin/bash
# (1) class words stored through the caches (build) / non-temporal (build_c) /
# before them (build_b): C2 device path A/B; (2) PMC fetch/write passes of the
# device path (build); (3) the records' D2H as a copy-engine copy
# (SID_D2H_NOCU=1) against the runtime's blit kernel: C2 PCIe-path value A/B
# and a short kernel trace.  Each step time-limited, the first failure ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O/r03pmc2
export TMPDIR=/tmp
REPS=3 BUILDS="build build_c build_b" timeout -k 10 600 bash tools/ab_builds.sh || { echo ab failed; exit 1; }
B="python3 $GRAFT_REPO_ROOT/bench.py --device-only --steps 2 --device-steps 2"
run() {
    local g=$1; shift
    ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/r03pmc2/pmc_$g -o p -- $B > $O/r03pmc2_$g.log 2>&1 )
}
run fetch FETCH_SIZE || exit $?
run write WRITE_SIZE || exit $?
python3 tools/pmc_summary.py $O/r03pmc2 --json $O/r03pmc2/summary.json > $O/r03pmc2/summary.txt || exit $?
for v in 1 0 1 0; do
  SID_D2H_NOCU=$v timeout -k 10 300 python3 -u bench.py --no-extras --steps 20 > $O/nocu_$v.json 2> $O/nocu_$v.err || { echo "nocu=$v failed"; tail -5 $O/nocu_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/nocu_$v.json')); print('nocu=$v', round(d['value']/1e8,3), round(d['ms_per_step'],2), round(d['pcie']['GBps_h2d'],1), round(d['pcie']['ceiling']['frac'],3))" | tee -a $O/nocu_ab.log
done
( cd /tmp && SID_D2H_NOCU=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/nocutrace -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-extras > $O/nocutrace.json 2> $O/nocutrace.log ) || { echo trace failed; tail $O/nocutrace.log; exit 1; }
head -8 $O/nocutrace/trace_kernel_stats.csv | cut -c1-150
