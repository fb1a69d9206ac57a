#!/bin/bash
# the cooperative parse under PMC (instruction mix, occupancy) and a kernel
# trace of the device path with it on
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
export SID_PARSE_COOP=1
B="python3 $GRAFT_REPO_ROOT/bench.py --device-only --steps 2 --device-steps 2"
( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/coop_pmc -o p -- $B > $O/coop_pmc.log 2>&1 ) || exit $?
( cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/coop_trace -o t -- $B > $O/coop_trace.log 2>&1 ) || exit $?
python3 - <<'PY'
import csv, os, collections
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out"
rows = list(csv.DictReader(open(O + "/coop_pmc/p_counter_collection.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in rows:
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")[-40:]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    if "parse" in k or "index" in k:
        print(k, {c: round(x / 8) for c, x in v.items()})
for r in list(csv.DictReader(open(O + "/coop_trace/t_kernel_stats.csv")))[:10]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:90]}")
PY
