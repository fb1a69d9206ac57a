#!/bin/bash
# round 6 A/B: the tile-parse tests on build/ (and on each BUILDS variant
# given in TEST_BUILDS), then tools/gpu/ab.sh over BUILDS for C2 and C5
. "$(dirname "$0")/common.sh"
TAG=${1:-r06}
for v in build ${TEST_BUILDS}; do
  SID_LIB_PATH=$PWD/$v/libsid.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
      tests/test_textpath_gpu.py tests/test_parse_stress_gpu.py tests/test_engine_gpu.py::test_tile_parse_slot_caps \
      > $O/pytest_tile_${TAG}_$v.log 2>&1 || { echo "tile tests failed on $v"; tail -30 $O/pytest_tile_${TAG}_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_tile_${TAG}_$v.log)"
done
REPS=${REPS:-3} tools/gpu/ab.sh ${TAG}_c2 || exit 1
[ -n "$C5" ] && { REPS=2 tools/gpu/ab.sh ${TAG}_c5 --config C5 || exit 1; }
exit 0
