#!/bin/bash
# A/B: current (build), intermediate arrays stored non-temporal (build_b)

set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
REPS=3 BUILDS="build build_b" timeout -k 10 900 bash tools/ab_builds.sh
