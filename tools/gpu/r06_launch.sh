#!/bin/bash
# round 6: the bench launcher tests, benches, stall/LDS counters of C2's device path
. "$(dirname "$0")/common.sh"
TAG=${1:-r06}
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/test_bench_launch.py \
    > $O/pytest_launch_$TAG.log 2>&1 || { echo launch failed; tail -30 $O/pytest_launch_$TAG.log; exit 1; }
tail -1 $O/pytest_launch_$TAG.log
tools/gpu/bench.sh $TAG C2 C3B || exit 1
PASSES="stall lds" tools/gpu/profile.sh ${TAG}_c2 || exit 1
exit 0
