#!/bin/bash
# A/B: current (build), more single-use reads non-temporal (build_b: masks, read-bases windows)

set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
REPS=3 BUILDS="build build_b" timeout -k 10 900 bash tools/ab_builds.sh
