#!/bin/bash
. tools/gpu/common.sh
for r in 1 2; do
  for cm in 0 4000; do
    timeout -k 10 200 python3 -u bench.py --device-only --steps 10 --chunk-mib $cm > $O/ab.json 2> $O/ab.err || { echo "failed"; tail -5 $O/ab.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/ab.json'))['device_path']
print('C2 chunk_mib=$cm', 'ms=%.3f' % d['ms_per_step'], {k: round(v, 3) for k, v in d['stages_ms'].items() if v})" | tee -a $O/ab_chunk.log
  done
done
for cm in 0 3584; do
  timeout -k 10 300 python3 -u bench.py --device-only --steps 5 --config C5 --chunk-mib $cm > $O/ab.json 2> $O/ab.err || { echo "failed"; tail -5 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/ab.json'))['device_path']
print('C5 chunk_mib=$cm', 'ms=%.3f' % d['ms_per_step'], {k: round(v, 3) for k, v in d['stages_ms'].items() if v})" | tee -a $O/ab_chunk.log
done
