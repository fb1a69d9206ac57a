#!/bin/bash
# A/B of build vs build_b on the C2 device path, then FETCH_SIZE / WRITE_SIZE
# per kernel for both (separate rocprofv3 passes)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
export TMPDIR=/tmp
REPS=${REPS:-2} bash tools/ab_builds.sh || exit $?
for v in build build_b; do
  for g in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && SID_LIB_PATH=$GRAFT_REPO_ROOT/$v/libsid.so timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d $O/abpmc_$v/pmc_$g -o p -- python3 $GRAFT_REPO_ROOT/bench.py --device-only --steps 2 --device-steps 2 > $O/abpmc_$v.$g.log 2>&1 ) || exit $?
  done
  echo $v; python3 tools/pmc_summary.py $O/abpmc_$v | grep -E "sid_local_put|sid_local_len|sid_parse_kernel|sid_index_count"
done
