#!/bin/bash
# kernel trace of the C2 bench (no extras) -> gpurun_out/c2trace/trace_kernel_stats.csv
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2trace -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-extras ${@} > $O/c2trace.log 2>&1 || exit $?
python3 - <<'PY'
import csv, os
p = os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out/c2trace/trace_kernel_stats.csv")
for r in list(csv.DictReader(open(p)))[:16]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:90]}")
PY
