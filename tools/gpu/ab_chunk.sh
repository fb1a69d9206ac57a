#!/bin/bash
# device-path A/B over builds x chunk sizes on one box:
#   CFG=C2 BUILDS="build build_b" CHUNKS="0 2048" REPS=2 tools/gpu/ab_chunk.sh TAG
. "$(dirname "$0")/common.sh"
TAG=${1:-run}
for r in $(seq ${REPS:-2}); do
  for v in ${BUILDS:-build}; do
    for cm in ${CHUNKS:-0}; do
      SID_LIB_PATH=$PWD/$v/libsid.so timeout -k 10 300 python3 -u bench.py --device-only --steps ${STEPS:-10} \
          --config ${CFG:-C2} --chunk-mib $cm > $O/ab.json 2> $O/ab.err || { echo "failed"; tail -5 $O/ab.err; exit 1; }
      python3 -c "
import json; d=json.load(open('$O/ab.json'))['device_path']
print('${CFG:-C2} $v chunk_mib=$cm', 'ms=%.3f' % d['ms_per_step'], {k: round(v, 3) for k, v in d['stages_ms'].items() if v})" | tee -a $O/ab_chunk_$TAG.log
    done
  done
done
