#!/bin/bash
# cooperative parse v2 (token-end mask only, per-line separator check, 4-window
# runs): parse tests in both modes, then device-path A/B (C2 and the C5 shard)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_parse_coop_gpu.py -x -q --timeout 400 --timeout-method thread > $O/coop_tests.log 2>&1 || { echo coop tests failed; grep -E "FAIL|Error|assert" $O/coop_tests.log | head -20; tail -40 $O/coop_tests.log; exit 1; }
tail -1 $O/coop_tests.log
for r in 1 2; do
    for c in 0 1; do
        SID_PARSE_COOP=$c timeout -k 10 200 python3 -u bench.py --device-only --steps 10 --device-steps 10 > $O/ab_c2_${c}_$r.json 2> $O/ab_c2_${c}_$r.err || { echo "bench coop=$c failed"; tail $O/ab_c2_${c}_$r.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/ab_c2_${c}_$r.json'))['device_path']; print('C2 coop=$c', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['stages_ms'].items()})"
    done
done
for c in 0 1; do
    SID_PARSE_COOP=$c timeout -k 10 300 python3 -u bench.py --config C5 --sites 62500000 --steps 3 > $O/ab_c5_$c.json 2> $O/ab_c5_$c.err || { echo "c5 coop=$c failed"; tail $O/ab_c5_$c.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/ab_c5_$c.json')); print('C5 shard coop=$c', round(d.get('ms_per_step'),3), {k: round(v,3) for k,v in d.get('device_path', {}).get('stages_ms').items()})"
done
