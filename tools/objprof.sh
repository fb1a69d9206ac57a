set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for t in 1 0; do
SID_MIX_TAB=$t timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/objp$t -o p -- python3 bench.py --method likelihood_ratio --cpu-sample 0 --no-e2e --steps 5 --warmup 1 > gpurun_out/objp$t.log 2>&1 || exit 1
done
