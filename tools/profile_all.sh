#!/bin/bash
# The round's profile set (one gpurun call): C2 and C3 benches under
# rocprofv3 (kernel trace + separate FETCH_SIZE / WRITE_SIZE passes), the CLI's
# device text path under a kernel trace, and the end-to-end CLI bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
PASSES="trace fetch write" PREFIX=local BENCH_ARGS="--steps 10 --warmup 2 --cpu-sample 0 --no-e2e" ./tools/profile_round.sh || exit 1
PASSES="trace fetch write" PREFIX=c3 BENCH_ARGS="--method likelihood_ratio --steps 5 --warmup 1 --cpu-sample 0 --no-e2e" ./tools/profile_round.sh || exit 1
python3 - <<'PY' || exit 1
import sys
sys.path.insert(0, ".")
import sid_amd
with open("/tmp/sid_cli20m.plp", "wb") as f:
    for lo in range(0, 20_000_000, 5_000_000):
        f.write(sid_amd.synth_text(2, 5_000_000, 30.0, first=lo))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cli_trace -o trace -- \
    ./build/sid /tmp/sid_cli20m.plp > /dev/null 2> $O/cli_trace.log || { echo "cli trace rc=$?"; exit 1; }
echo "cli trace ok"
SITES=${E2E_SITES:-50000000} ./tools/e2e_bench.sh || exit 1
