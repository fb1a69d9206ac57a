#!/bin/bash
# the PCIe-inclusive C2 step: build vs build_b, interleaved, + engine tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_engine_gpu.py tests/test_cli_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_e2e.log 2>&1 || { echo tests failed; tail -30 $O/pytest_e2e.log; exit 1; }
tail -1 $O/pytest_e2e.log
for r in 1 2; do for v in build build_b; do
  SID_LIB_PATH=$PWD/$v/libsid.so timeout -k 10 300 python3 -u bench.py --no-extras --steps 10 --device-steps 2 > $O/e2e_$v.json 2> $O/e2e_$v.err || { echo fail $v; tail $O/e2e_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/e2e_$v.json')); print('$v', d['value'], d['ms_per_step'], d['pcie']['ingest_s'], d['pcie']['chunks'])"
done; done
