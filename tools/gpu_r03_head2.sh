#!/bin/bash
# round-3 re-entry check at HEAD (tools/gpu_r03_head.sh), then the CLI exit A/B
# (tools/cli_exit_ab.py); each step time-limited, the first failure ends it
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
bash tools/gpu_r03_head.sh || exit 1
timeout -k 10 300 python3 -u tools/cli_exit_ab.py 50000000 3 > $O/cli_exit_ab.jsonl 2> $O/cli_exit_ab.err || { echo cli ab failed; tail $O/cli_exit_ab.err; exit 1; }
cat $O/cli_exit_ab.jsonl
