#!/bin/bash
# C4 and C5 bench lines at HEAD (each time-limited, the first failure ends it)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u bench.py --config C4 --steps 3 > $O/bench_c4.json 2> $O/bench_c4.err || { echo c4 failed; tail $O/bench_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c4.json')); print('C4', d['value'], d['ms_per_step'], d['generator'], d['device_path']['stages_ms'])"
timeout -k 10 600 python3 -u bench.py --config C5 --steps 2 > $O/bench_c5.json 2> $O/bench_c5.err || { echo c5 failed; tail $O/bench_c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c5.json')); print('C5', d['value'], d['ms_per_step'], d['generator'], d['device_path']['stages_ms'])"
