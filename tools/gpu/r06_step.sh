#!/bin/bash
# round 6 working steps (one gpurun call): tile-parse tests on the current
# build, the A/B of build_prev vs build, the bench launcher tests, benches
. "$(dirname "$0")/common.sh"
TAG=${1:-r06}
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_textpath_gpu.py \
    tests/test_parse_stress_gpu.py tests/test_engine_gpu.py::test_tile_parse_slot_caps \
    tests/test_engine_gpu.py::test_tile_parse_recovers_on_a_reused_engine > $O/pytest_tile_$TAG.log 2>&1 \
    || { echo "tile tests failed"; tail -30 $O/pytest_tile_$TAG.log; exit 1; }
tail -1 $O/pytest_tile_$TAG.log
BUILDS="build_prev build" REPS=3 tools/gpu/ab.sh ${TAG}_c2 || exit 1
BUILDS="build_prev build" REPS=2 tools/gpu/ab.sh ${TAG}_c5 --config C5 || exit 1
if [ -n "$LAUNCH" ]; then
  timeout -k 10 900 python3 -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/test_bench_launch.py \
      > $O/pytest_launch_$TAG.log 2>&1 || { echo launch failed; tail -30 $O/pytest_launch_$TAG.log; exit 1; }
  tail -1 $O/pytest_launch_$TAG.log
fi
[ -n "$BENCH" ] && tools/gpu/bench.sh $TAG $BENCH
exit 0
