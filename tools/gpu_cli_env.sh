#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u tools/debug/cli_env_probe.py | tee gpurun_out/cli_env.jsonl
