#!/bin/bash
# the whole GPU suite, then the C2 device path three times and C3 once
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo tests failed; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for r in 1 2 3; do
    timeout -k 10 200 python3 -u bench.py --device-only --steps 10 --device-steps 20 > $O/dev_c2_$r.json 2> $O/dev_c2_$r.err || { echo "bench failed"; tail $O/dev_c2_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/dev_c2_$r.json'))['device_path']; print('C2 device', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['stages_ms'].items()})"
done
timeout -k 10 200 python3 -u bench.py --config C3 --device-only --steps 10 --device-steps 20 > $O/dev_c3.json 2> $O/dev_c3.err || { echo "bench c3 failed"; tail $O/dev_c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/dev_c3.json'))['device_path']; print('C3 device', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['stages_ms'].items()})"
