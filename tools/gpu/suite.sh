#!/bin/bash
# the GPU test suite (pytest -m gpu, or the files / node ids given), then the
# smoke test of __graft_entry__; logs gpurun_out/pytest_gpu_<TAG>.log,
# gpurun_out/smoke_<TAG>.txt.   usage: tools/gpu/suite.sh TAG [pytest targets]
. "$(dirname "$0")/common.sh"
TAG=${1:-run}; shift
T=${*:-tests}
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu $T \
    > $O/pytest_gpu_$TAG.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" $O/pytest_gpu_$TAG.log | head; tail -5 $O/pytest_gpu_$TAG.log; exit 1; }
tail -1 $O/pytest_gpu_$TAG.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.txt 2>&1 || { echo "smoke failed"; tail $O/smoke_$TAG.txt; exit 1; }
tail -2 $O/smoke_$TAG.txt
