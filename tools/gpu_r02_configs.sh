#!/bin/bash
# C3 / C4 / C5 bench lines on one GPU and a 2-rank rehearsal (gloo, shared GPU)
# of the C2 and C3 multi-rank paths; each step time-limited, the first failure ends it
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
run() {  # name, timeout, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed rc=$?"; tail -8 $O/$n.err; exit 1; }
  python3 -c "
import json
d = json.loads([l for l in open('$O/$n.json') if l.startswith('{')][-1])
print('$n', 'value=%.4g' % d['value'], 'ms=%.2f' % d['ms_per_step'], d.get('n_gpus'), {k: round(v, 2) for k, v in d['stages_ms'].items()})"
}
run bench_c3 300 python3 -u bench.py --config C3 --steps 10 --no-cpu
run bench_c4 400 python3 -u bench.py --config C4 --steps 2 --warmup 1
run bench_c5 400 python3 -u bench.py --config C5 --steps 2 --warmup 1
run bench_2r_c2 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --allow-shared-gpu --backend gloo
run bench_2r_c3 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config C3 --steps 5 --warmup 2 --allow-shared-gpu --backend gloo
