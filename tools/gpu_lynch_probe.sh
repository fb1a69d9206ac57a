#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/debug/lynch_stress_probe.py 2>&1 | head -12
timeout -k 10 300 python3 -u tools/debug/lynch_points_probe.py
timeout -k 10 300 python3 -u tools/debug/stress_probe.py build 2>&1 | grep likeli
