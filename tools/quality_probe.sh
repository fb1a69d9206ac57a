#!/bin/bash
# -m quality: parity tests, then the CLI on a 20M-site 7-column 30x file
# under a kernel trace (per-kernel durations) -- measurement only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
SITES=${SITES:-20000000}
F=/tmp/sid_q_${SITES}_${DEPTH:-30}.plp
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python3 -u -m pytest tests/test_quality_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_quality.log 2>&1 || { echo "tests rc=$?"; tail -20 $O/pytest_quality.log; exit 1; }
echo tests ok
fi
python3 - <<PY || exit 1
import sys
sys.path.insert(0, ".")
import sid_amd
with open("$F", "wb") as f:
    for lo in range(0, $SITES, 5_000_000):
        f.write(sid_amd.synth_text(2, min(5_000_000, $SITES - lo), ${DEPTH:-30.0}, first=lo, mapq=True))
PY
cat $F > /dev/null
for rep in 1 2; do
  timeout -k 10 300 ${SIDBIN:-./build/sid} --stats -m quality $F > /dev/null 2> $O/q_stats.txt || { echo "sid rc=$?"; tail -3 $O/q_stats.txt; exit 1; }
  tail -1 $O/q_stats.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/q_trace -o trace -- \
    ${SIDBIN:-./build/sid} -m quality $F > /dev/null 2> $O/q_trace.log || { echo "trace rc=$?"; exit 1; }
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/q_trace/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Name"][:70], r["Calls"], r["AverageNs"])
PY
