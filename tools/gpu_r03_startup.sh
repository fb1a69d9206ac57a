#!/bin/bash
# CLI start-up pieces (tools/debug/startup_probe.cpp, 3 runs) and the device
# path's host overhead (SID_ENGINE_TIMING), each step time-limited
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 60 ./build/startup_probe >> $O/startup_probe.jsonl 2>&1 || { echo probe failed; cat $O/startup_probe.jsonl; exit 1; }
done
cat $O/startup_probe.jsonl
SID_ENGINE_TIMING=1 timeout -k 10 300 python3 -u bench.py --device-only --steps 10 > $O/dev_timing.json 2> $O/dev_timing.err || { echo dev failed; tail $O/dev_timing.err; exit 1; }
grep engine_phase $O/dev_timing.err | tail -6
python3 -c "import json; d=json.load(open('$O/dev_timing.json')); print(d['ms_per_step'], d['device_path']['stages_ms'])"
