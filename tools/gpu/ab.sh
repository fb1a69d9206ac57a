#!/bin/bash
# A/B of builds of the same sources (make BUILD=build_b EXTRA=-D...), the
# device path (bench.py --device-only) interleaved on one box, REPS rounds:
# gpurun_out/ab_<TAG>.log.   usage: BUILDS="build build_b" tools/gpu/ab.sh TAG [bench args]
. "$(dirname "$0")/common.sh"
TAG=${1:-run}; shift
for r in $(seq ${REPS:-3}); do
  for v in ${BUILDS:-build build_b}; do
    SID_LIB_PATH=$PWD/$v/libsid.so timeout -k 10 200 python3 -u bench.py --device-only --steps 10 "$@" \
        > $O/ab.json 2> $O/ab.err || { echo "$v failed"; tail -5 $O/ab.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/ab.json'))['device_path']
print('$v', 'ms=%.3f' % d['ms_per_step'], {k: round(v, 3) for k, v in d['stages_ms'].items()})" | tee -a $O/ab_$TAG.log
  done
done
