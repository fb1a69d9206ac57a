#!/bin/bash
# engine + CLI parity after a formatter change, then an A/B of build vs build_b
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_engine_gpu.py tests/test_cli_gpu.py tests/test_textpath_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_c.log 2>&1 || { echo tests failed; grep -E "FAIL|Error|assert" $O/pytest_c.log | head -20; tail -30 $O/pytest_c.log; exit 1; }
tail -2 $O/pytest_c.log
REPS=${REPS:-2} bash tools/ab_builds.sh
