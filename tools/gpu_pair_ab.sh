#!/bin/bash
# the fused parse's header pair as one 16-B non-temporal store (build) against
# two 8-B stores (build_c, HEAD): C2 device path A/B, then PMC fetch/write
# passes of the device path for build (each step time-limited)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O/r03pmc4
export TMPDIR=/tmp
REPS=3 BUILDS="build build_c" timeout -k 10 600 bash tools/ab_builds.sh || { echo ab failed; exit 1; }
B="python3 $GRAFT_REPO_ROOT/bench.py --device-only --steps 2 --device-steps 2"
run() {
    local g=$1; shift
    ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/r03pmc4/pmc_$g -o p -- $B > $O/r03pmc4_$g.log 2>&1 )
}
run fetch FETCH_SIZE || exit $?
run write WRITE_SIZE || exit $?
python3 tools/pmc_summary.py $O/r03pmc4 --json $O/r03pmc4/summary.json > $O/r03pmc4/summary.txt || exit $?
python3 - <<'PY'
import json, os
d = json.load(open(os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out/r03pmc4/summary.json")))
for k in ("sid_parse_len_kernel", "sid_local_put_kernel", "sid_index_emit_kernel"):
    r = d[k]
    print(k, "fetch %.1f write %.1f B/site" % (r["FETCH_SIZE"] * 2048 / 25e6, r["WRITE_SIZE"] * 1024 / 25e6))
PY
