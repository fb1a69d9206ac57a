#!/bin/bash
# C2 PCIe leg: chunk size / device text buffers sweep
cd $GRAFT_REPO_ROOT
for cfg in "128 0" "64 0" "256 0" "32 0" "128 4" "64 6" "128 0"; do
  set -- $cfg
  timeout -k 10 240 python3 -u bench.py --no-extras --steps 10 --warmup 2 --pcie-chunk-mib $1 --slots $2 > gpurun_out/pc.json 2> gpurun_out/pc.err || { echo "fail $cfg"; tail -3 gpurun_out/pc.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/pc.json')); print('chunk_mib=$1 slots=$2', 'value=%.4e' % d['value'], 'ms=%.2f' % d['ms_per_step'])" | tee -a gpurun_out/pcie_sweep.log
done
