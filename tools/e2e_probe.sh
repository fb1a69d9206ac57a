#!/bin/bash
# e2e CLI variants on one 50M-site 30x file (page cache, CSV to /dev/null),
# with the CLI's phase timers (SID_TEXT_TIMING) -- measurement only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
SITES=${SITES:-50000000}
F=/tmp/sid_probe_${SITES}.plp
python3 - <<PY || exit 1
import sys
sys.path.insert(0, ".")
import sid_amd
with open("$F", "wb") as f:
    for lo in range(0, $SITES, 5_000_000):
        f.write(sid_amd.synth_text(2, min(5_000_000, $SITES - lo), 30.0, first=lo))
PY
cat $F > /dev/null
run() {   # tag, env...
  tag=$1; shift
  for rep in 1 2; do
    a=$(date +%s.%N)
    env "$@" SID_TEXT_TIMING=1 timeout -k 10 300 ./build/sid --stats $F > /dev/null 2> $O/probe_$tag.err || { echo "$tag rc=$?"; tail -3 $O/probe_$tag.err; exit 1; }
    b=$(date +%s.%N)
    echo "{\"tag\": \"$tag\", \"rep\": $rep, \"wall_s\": $(python3 -c "print('%.4f' % ($b - $a))"), \"lines\": [$(paste -sd, $O/probe_$tag.err)]}" | tee -a $O/e2e_probe.jsonl
  done
}
for v in ${VARIANTS:-default default}; do
  case $v in
    default) run default ;;
    fd) run fd SID_READ_FD=1 ;;
    nosdma) run nosdma HSA_ENABLE_SDMA=0 ;;
    piece1k) run piece1k SID_FMT_PIECE_BLOCKS=1024 ;;
    piece256) run piece256 SID_FMT_PIECE_BLOCKS=256 ;;
  esac
done
