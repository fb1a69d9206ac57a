#!/bin/bash
# A/B/C of the -m local writer variants (build: OR-ed pieces, build_b: LDS
# byte stores, build_c: flat byte stores), each checked against the oracle first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
for v in ${BUILDS:-build build_b build_c}; do
  SID_LIB_PATH=$PWD/$v/libsid.so timeout -k 10 300 python3 -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "sources or long_chrom or lanes" > $O/pytest_$v.log 2>&1 || { echo "$v tests failed"; tail -20 $O/pytest_$v.log; exit 1; }
  tail -1 $O/pytest_$v.log
done
BUILDS="${BUILDS:-build build_b build_c}" REPS=${REPS:-3} bash tools/ab_builds.sh
