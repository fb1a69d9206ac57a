#!/bin/bash
# A/B of environment settings on the C2 bench (no extras): SWEEP="NAME=v1 NAME=v2 ..."
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
for kv in $SWEEP; do
  env $kv timeout -k 10 200 python3 -u bench.py --no-extras "$@" > $O/sweep.json 2> $O/sweep.err || { echo "$kv failed"; tail -5 $O/sweep.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/sweep.json'))
print('$kv', 'value=%.4g' % d['value'], 'ms=%.3f' % d['ms_per_step'], {k: round(v, 3) for k, v in d['stages_ms'].items()})" | tee -a $O/sweep.log
done
