#!/bin/bash
# A/B of builds on one box: BUILDS (default "build build_b"), the C2 device
# path (bench.py --device-only) interleaved, REPS rounds
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
for r in $(seq ${REPS:-3}); do
  for v in ${BUILDS:-build build_b}; do
    SID_LIB_PATH=$PWD/$v/libsid.so timeout -k 10 200 python3 -u bench.py --device-only --steps 10 "$@" > $O/ab.json 2> $O/ab.err || { echo "$v failed"; tail -5 $O/ab.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/ab.json'))['device_path']
print('$v', 'ms=%.3f' % d['ms_per_step'], {k: round(v, 3) for k, v in d['stages_ms'].items()})" | tee -a $O/ab.log
  done
done
