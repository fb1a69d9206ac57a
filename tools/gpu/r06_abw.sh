#!/bin/bash
# round 6: the GPU tests that cover the writers and the tile parse on build/,
# then the A/B over BUILDS (C2 and C5)
. "$(dirname "$0")/common.sh"
TAG=${1:-r06}
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_textpath_gpu.py \
    tests/test_parse_stress_gpu.py tests/test_engine_gpu.py tests/test_cli_gpu.py tests/test_local_gpu.py \
    tests/test_lynch_gpu.py > $O/pytest_w_$TAG.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest_w_$TAG.log; exit 1; }
tail -1 $O/pytest_w_$TAG.log
REPS=${REPS:-3} tools/gpu/ab.sh ${TAG}_c2 || exit 1
[ -n "$C5" ] && { REPS=2 tools/gpu/ab.sh ${TAG}_c5 --config C5 || exit 1; }
[ -n "$C3" ] && { REPS=2 tools/gpu/ab.sh ${TAG}_c3 --config C3 || exit 1; }
exit 0
