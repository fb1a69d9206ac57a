set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
for v in "1 1" "1 0"; do set -- $v
 SID_LYNCH_TIMING=1 SID_NM_DEVICE=$1 SID_NM_LOOKAHEAD=$2 timeout -k 10 120 python3 bench.py --method likelihood_ratio --cpu-sample 0 --no-e2e --steps 5 > $O/nm_c3_$1_$2.json 2>$O/nm_c3_$1_$2.err || exit 1
done
