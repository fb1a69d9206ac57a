#!/bin/bash
# A/B of builds on one box: BUILDS (default "build build_b"), C2 bench (no
# extras) interleaved, REPS rounds
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
for r in $(seq ${REPS:-3}); do
  for v in ${BUILDS:-build build_b}; do
    SID_LIB_PATH=$PWD/$v/libsid.so timeout -k 10 200 python3 -u bench.py --no-extras "$@" > $O/ab.json 2> $O/ab.err || { echo "$v failed"; tail -5 $O/ab.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/ab.json'))
print('$v', 'value=%.4g' % d['value'], 'ms=%.3f' % d['ms_per_step'], {k: round(v, 3) for k, v in d['stages_ms'].items()})" | tee -a $O/ab.log
  done
done
