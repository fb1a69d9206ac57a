#!/bin/bash
# PCIe-path chunk size x device text slots, C2 (no extras)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
for r in 1 2; do
for cfg in "128 3" "128 6" "256 3" "256 4" "64 6"; do
  set -- $cfg
  timeout -k 10 300 python3 -u bench.py --no-extras --steps 10 --device-steps 2 --pcie-chunk-mib $1 --slots $2 > $O/sw.json 2> $O/sw.err || { echo fail $cfg; tail $O/sw.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/sw.json')); print('chunk $1 MiB slots $2', round(d['ms_per_step'], 2), d['pcie']['chunks'])"
done; done
