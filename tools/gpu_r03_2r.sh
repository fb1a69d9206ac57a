#!/bin/bash
# --gpus N without torchrun: the refusal on a 1-GPU box, then the 2-rank
# rehearsal on one GPU (C2, C3) -- the spawn path the driver's N-GPU runs take
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
if timeout -k 10 120 python3 -u bench.py --gpus 2 --no-cpu > $O/refuse.out 2> $O/refuse.err; then echo "NOT refused"; exit 1; fi
echo "refused: $(tail -1 $O/refuse.err)"
timeout -k 10 500 python3 -u bench.py --gpus 2 --allow-shared-gpu --no-cpu > $O/bench_2r_c2.json 2> $O/bench_2r_c2.err || { echo 2r failed; tail $O/bench_2r_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_2r_c2.json')); print('2r C2', d['value'], d['ms_per_step'], d['n_gpus'], d['config']['ranks'], d['config']['oversubscribed'], d['config']['rccl_world'])"
timeout -k 10 500 python3 -u bench.py --gpus 2 --allow-shared-gpu --config C3 --no-cpu > $O/bench_2r_c3.json 2> $O/bench_2r_c3.err || { echo 2r c3 failed; tail $O/bench_2r_c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_2r_c3.json')); print('2r C3', d['value'], d['ms_per_step'], d['n_gpus'], d['config']['ranks'], d['config']['oversubscribed'], d['config']['rccl_world'], d.get('estimate'))"
