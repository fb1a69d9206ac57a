#!/bin/bash
# -m local record lengths out of the parse: the GPU suite, then an A/B of the
# device path against the separate length kernel (SID_PARSE_LEN=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_cli_gpu.py tests/test_engine_gpu.py tests/test_parse_coop_gpu.py tests/test_benchpath_gpu.py -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo tests failed; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for r in 1 2; do
    for c in 0 1; do
        SID_PARSE_LEN=$c timeout -k 10 200 python3 -u bench.py --device-only --steps 10 --device-steps 10 > $O/ab_len_${c}_$r.json 2> $O/ab_len_${c}_$r.err || { echo "bench len=$c failed"; tail $O/ab_len_${c}_$r.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/ab_len_${c}_$r.json'))['device_path']; print('C2 parse_len=$c', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['stages_ms'].items()})"
    done
done
