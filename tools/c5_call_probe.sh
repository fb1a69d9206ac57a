#!/bin/bash
# C5 (200x) call-kernel probe: kernel trace of a 20M-site C5 run per env variant
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$PWD/gpurun_out; mkdir -p $O
export TMPDIR=/tmp
while read -r tag envs; do
  [ -z "$tag" ] && continue
  (cd /tmp && env $envs timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5p_$tag -o t -- python3 $GRAFT_REPO_ROOT/bench.py --config C5 --sites 20000000 --steps 1 --warmup 1 --no-extras > $O/c5p_$tag.log 2>&1) || { echo "$tag failed"; tail -5 $O/c5p_$tag.log; exit 1; }
  python3 - "$O/c5p_$tag/t_kernel_stats.csv" "$tag" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "local" in r["Name"] or "fixup" in r["Name"]:
        print(sys.argv[2], f"{int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:70]}")
PY
done <<< "$VARIANTS"
