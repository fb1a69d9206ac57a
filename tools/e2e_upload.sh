#!/bin/bash
# CLI e2e on one 50M-site 30x file (page cache, CSV to /dev/null) under the
# upload variants (SID_UPLOAD = staged | map | pageable) -- measurement only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
SITES=${SITES:-50000000}
F=/tmp/sid_up_${SITES}.plp
python3 - <<PY || exit 1
import sys
sys.path.insert(0, ".")
import sid_amd
with open("$F", "wb") as f:
    for lo in range(0, $SITES, 5_000_000):
        f.write(sid_amd.synth_text(2, min(5_000_000, $SITES - lo), 30.0, first=lo))
PY
cat $F > /dev/null
for v in ${VARIANTS:-staged pageable map staged}; do
  for rep in 1 2; do
    a=$(date +%s.%N)
    SID_ENGINE_TIMING=1 SID_UPLOAD=$v timeout -k 10 300 ./build/sid --stats $F > /dev/null 2> $O/up_$v.err || { echo "$v rc=$?"; tail -3 $O/up_$v.err; exit 1; }
    b=$(date +%s.%N)
    echo "{\"upload\": \"$v\", \"rep\": $rep, \"wall_s\": $(python3 -c "print('%.4f' % ($b - $a))"), \"stats\": $(tail -1 $O/up_$v.err)}" | tee -a $O/e2e_upload.jsonl
  done
done
