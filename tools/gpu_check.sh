#!/bin/bash
# GPU check: the whole -m gpu suite, then the C2 bench (no extras) and a C5 pass.
# usage: tools/gpu_check.sh [pytest selection]   (outputs under gpurun_out/)
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
SEL=${1:-tests}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $SEL > $O/gputests.log 2>&1
rc=$?
tail -5 $O/gputests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; grep -E "FAILED|Error|assert" $O/gputests.log | head -20; exit $rc; fi
timeout -k 10 300 python -u bench.py --no-extras > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
timeout -k 10 300 python -u bench.py --config C5 --steps 1 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
python3 - <<'PY'
import json
for f in ("gpurun_out/bench_c2.json", "gpurun_out/bench_c5.json"):
    d = json.load(open(f))
    print(f, f"value={d['value']:.4g} ms/step={d['ms_per_step']:.2f}", {k: round(v, 3) for k, v in d["stages_ms"].items()},
          "roof", d["roofline"]["kernel"], round(d["roofline"]["frac"], 3))
PY
