#!/bin/bash
# one iteration: the text-path / engine / CLI GPU tests, then the C2 bench (no
# extras) and its kernel trace.  TESTS overrides the test selection.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
T=${TESTS:-"tests/test_textpath_gpu.py tests/test_engine_gpu.py tests/test_cli_gpu.py"}
if [ "$T" != "none" ]; then
timeout -k 10 600 python3 -u -m pytest $T -x -q --timeout 300 --timeout-method thread > $O/pytest_iter.log 2>&1 || { echo tests failed; tail -40 $O/pytest_iter.log; exit 1; }
tail -2 $O/pytest_iter.log
fi
bash tools/gpu_perf.sh "$@"
