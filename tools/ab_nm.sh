# A/B of the Lynch estimate: device-resident (cooperative kernel) vs host-driven
# Nelder-Mead, with and without lookahead.  Run on the GPU box via gpurun.
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lynch_gpu.py -m gpu > $O/nm_tests.log 2>&1 || { echo tests failed; tail -30 $O/nm_tests.log; exit 1; }
for v in "1 1" "1 0" "0 1"; do set -- $v
 SID_LYNCH_TIMING=1 SID_NM_DEVICE=$1 SID_NM_LOOKAHEAD=$2 timeout -k 10 120 python3 bench.py --method likelihood_ratio --cpu-sample 0 --no-e2e > $O/nm_c3_$1_$2.json 2>$O/nm_c3_$1_$2.err || exit 1
done
