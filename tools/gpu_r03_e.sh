#!/bin/bash
# Fused Lynch formatter: engine / CLI / Lynch GPU tests and the full-size C3
# bench-path parity, then C3's device path with the fusion on and off
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_engine_gpu.py tests/test_cli_gpu.py tests/test_lynch_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_e.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest_e.log; exit 1; }
tail -1 $O/pytest_e.log
timeout -k 10 400 python3 -u -m pytest tests/test_benchpath_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k c3 > $O/pytest_e_c3.log 2>&1 || { echo "c3 failed"; tail -30 $O/pytest_e_c3.log; exit 1; }
tail -1 $O/pytest_e_c3.log
for f in 1 0 1 0; do
  SID_LYNCH_FUSED=$f timeout -k 10 200 python3 -u bench.py --config C3 --device-only --steps 10 --warmup 2 > $O/bench_c3_f$f.json 2> $O/bench_c3_f$f.err || { echo "bench f=$f failed"; tail -20 $O/bench_c3_f$f.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('$O/bench_c3_f$f.json').read().strip().splitlines()[-1])
dp=d.get('device_path',d)
print('fused=$f', d.get('value'), json.dumps(dp.get('stages_ms', dp.get('stages')))[:400])
"
done
