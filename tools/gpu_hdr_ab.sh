#!/bin/bash
# header A/B: 32-byte unaligned header (build), the same without the 64-VGPR
# cap (build_b), the 48-byte aligned header (build_c); parse tests first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_parse_coop_gpu.py tests/test_textpath_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 500 --timeout-method thread > $O/hdr_tests.log 2>&1 || { echo tests failed; grep -E "FAIL|Error|assert" $O/hdr_tests.log | head; tail -20 $O/hdr_tests.log; exit 1; }
tail -1 $O/hdr_tests.log
REPS=2 BUILDS="build build_b build_c" timeout -k 10 900 bash tools/ab_builds.sh
