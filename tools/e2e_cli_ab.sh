#!/bin/bash
# CLI e2e A/B on one 50M-site 30x file (page cache, CSV to /dev/null): each
# variant is "tag VAR=value ..." (environment), two runs each, engine timing on
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
SITES=${SITES:-50000000}
F=/tmp/sid_ab_${SITES}.plp
python3 - <<PY || exit 1
import sys
sys.path.insert(0, ".")
import sid_amd
with open("$F", "wb") as f:
    for lo in range(0, $SITES, 5_000_000):
        f.write(sid_amd.synth_text(2, min(5_000_000, $SITES - lo), 30.0, first=lo))
PY
cat $F > /dev/null
while read -r tag envs; do
  [ -z "$tag" ] && continue
  for rep in 1 2; do
    a=$(date +%s.%N)
    env SID_ENGINE_TIMING=1 $envs timeout -k 10 300 ./build/sid --stats $FLAGS $F > /dev/null 2> $O/ab_$tag.err || { echo "$tag rc=$?"; tail -3 $O/ab_$tag.err; exit 1; }
    b=$(date +%s.%N)
    echo "{\"tag\": \"$tag\", \"rep\": $rep, \"wall_s\": $(python3 -c "print('%.4f' % ($b - $a))"), \"lines\": [$(paste -sd, $O/ab_$tag.err)]}" | tee -a $O/e2e_ab.jsonl
  done
done <<< "$VARIANTS"
