# Lynch-path tests + C3 bench A/B (phase timing on stderr); gpurun helper.
# NM_VARIANTS: "DEVICE_LOOKAHEAD_MIXTAB ..." e.g. "0_1_1 0_1_0"
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
if [ -z "$NO_TESTS" ]; then
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lynch_gpu.py -m gpu > $O/nm_tests.log 2>&1 || { echo tests failed; tail -40 $O/nm_tests.log; exit 1; }
tail -1 $O/nm_tests.log
fi
for r in 1 2; do
for v in ${NM_VARIANTS:-"0_1_1"}; do IFS=_ read d l t <<< "$v"
 SID_LYNCH_TIMING=1 SID_NM_DEVICE=$d SID_NM_LOOKAHEAD=$l SID_MIX_TAB=$t timeout -k 10 120 python3 bench.py --method likelihood_ratio --cpu-sample 0 --no-e2e > $O/nm_c3_${v}_$r.json 2>$O/nm_c3_${v}_$r.err || exit 1
done
done
