#!/bin/bash
# A/B of environment settings on the same build: bench.py (its device path)
# interleaved on one box, REPS rounds: gpurun_out/envab_<TAG>.log.
# usage: ENVS="SID_X=1 SID_X=0" tools/gpu/env_ab.sh TAG [bench args]
. "$(dirname "$0")/common.sh"
TAG=${1:-run}; shift
for r in $(seq ${REPS:-2}); do
  for kv in ${ENVS:?ENVS=\"K=V K=V\"}; do
    env "$kv" timeout -k 10 300 python3 -u bench.py --device-only --steps 10 --no-cpu "$@" \
        > $O/envab.json 2> $O/envab.err || { echo "$kv failed"; tail -5 $O/envab.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/envab.json')); p=d['device_path']
print('$kv', 'value %.4g' % d['value'], 'ms=%.3f' % p['ms_per_step'], {k: round(v, 3) for k, v in p['stages_ms'].items()})" | tee -a $O/envab_$TAG.log
  done
done
