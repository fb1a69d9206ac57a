#!/bin/bash
# the PCIe-inclusive C2 step with HSA_ENABLE_SDMA as bench.py now sets it (1)
# and as the runtime defaults it (unset: bench.py's setdefault is bypassed by
# an explicit empty... so compare 1 against 0 and against the probe), + CLI wall
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
for v in 1 0; do
  HSA_ENABLE_SDMA=$v timeout -k 10 300 python3 -u bench.py --no-cpu --steps 10 --device-steps 4 > $O/e2e_sdma$v.json 2> $O/e2e_sdma$v.err || { echo fail $v; tail $O/e2e_sdma$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/e2e_sdma$v.json')); print('SDMA=$v', d['value'], d['ms_per_step'], d['pcie']['ingest_s'], d['cli']['wall_s'], d['cli']['cli_stats'].get('emit_s'))"
done
