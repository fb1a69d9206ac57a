# Kernel + HIP API + memcopy timeline of a short C3 bench run (no PMC), for
# the gaps between the step's kernels.  Output under gpurun_out/c3tl.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv -d gpurun_out/c3tl -o tl -- \
    python3 bench.py --method likelihood_ratio --steps 3 --warmup 1 --cpu-sample 0 --no-e2e > gpurun_out/c3tl.log 2>&1
