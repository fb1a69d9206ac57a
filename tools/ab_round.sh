set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_local_gpu.py tests/test_lynch_gpu.py -m gpu > $O/ab_tests.log 2>&1 || { echo tests failed; exit 1; }
timeout -k 10 120 python3 bench.py --cpu-sample 0 --no-e2e > $O/ab_local.json 2>$O/ab_local.err || exit 1
for v in "1 4096" "2 1024" "1 1024" "2 4096" "1 8192"; do set -- $v
 SID_LOOKUP_UNROLL=$1 SID_LOOKUP_GRID=$2 timeout -k 10 120 python3 bench.py --method likelihood_ratio --cpu-sample 0 --no-e2e > $O/ab_c3_$1_$2.json 2>$O/ab_c3.err || exit 1
done
