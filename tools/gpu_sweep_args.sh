#!/bin/bash
# A/B of bench.py argument sets on one box: ARGSETS="--lanes 1;--lanes 2;..." (no extras)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
IFS=';' read -ra SETS <<< "$ARGSETS"
for args in "${SETS[@]}"; do
  timeout -k 10 300 python3 -u bench.py --no-extras $args > $O/sweep.json 2> $O/sweep.err || { echo "[$args] failed"; tail -5 $O/sweep.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/sweep.json'))
print('[$args]', 'value=%.4g' % d['value'], 'ms=%.3f' % d['ms_per_step'], {k: round(v, 3) for k, v in d['stages_ms'].items()})" | tee -a $O/sweep.log
done
