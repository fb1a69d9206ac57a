#!/bin/bash
# after the parity fixes (long double denormal shift, emulated Lynch mixture,
# oracle BH by std::sort) with the cooperative parse opt-in: the parse tests
# in both modes, the whole GPU suite, the C2 bench line, the PCIe ceiling
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo tests failed; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python3 -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo bench failed; tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c2.json')); print('C2', d['value'], d['ms_per_step'], d['pcie']['GBps_h2d'], d['device_path']['ms_per_step'], {k: round(v,3) for k,v in d['device_path']['stages_ms'].items()}, d['roofline']['frac'], d['roofline']['kernel'])"
g++ -O2 -o /tmp/pcie_probe tools/debug/pcie_probe.cpp -I/opt/rocm/include -L/opt/rocm/lib -lamdhip64 -D__HIP_PLATFORM_AMD__ 2>/dev/null || hipcc -O2 -o /tmp/pcie_probe tools/debug/pcie_probe.cpp || exit 1
timeout -k 10 120 /tmp/pcie_probe > $O/pcie_probe.jsonl 2>&1 || { echo probe failed; cat $O/pcie_probe.jsonl; exit 1; }
cat $O/pcie_probe.jsonl
