#!/bin/bash
# -m local writer A/B: current (build), non-temporal record stores (build_b),
# 6 waves per SIMD (build_c)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
REPS=3 BUILDS="build build_b build_c" timeout -k 10 900 bash tools/ab_builds.sh
