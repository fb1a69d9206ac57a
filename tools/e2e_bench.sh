#!/bin/bash
# End-to-end CLI throughput on synthetic pileup text (file in page cache,
# CSV to /dev/null): the device text path, the host parse/emit path, and the
# oracle CLI (reference restated, 1 thread) on a bounded sample.
# usage: SITES=50000000 SAMPLE=2000000 tools/e2e_bench.sh   (on the GPU box)
#        FLAGS="-m quality" MAPQ=1 ... (7-column text for the quality method)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
SITES=${SITES:-50000000}
SAMPLE=${SAMPLE:-2000000}
DEPTH=${DEPTH:-30}
SEED=${SEED:-2}
MAPQ=${MAPQ:-0}
FLAGS=${FLAGS:-}
F=/tmp/sid_e2e_${SEED}_${SITES}_${DEPTH}_${MAPQ}.plp
S=/tmp/sid_e2e_${SEED}_${SAMPLE}_${DEPTH}_${MAPQ}.plp
python3 - <<PY || exit 1
import os, sys
sys.path.insert(0, ".")
import sid_amd
for path, n in (("$F", $SITES), ("$S", $SAMPLE)):
    if not os.path.exists(path):
        with open(path, "wb") as f:
            step = 5_000_000
            for lo in range(0, n, step):
                f.write(sid_amd.synth_text($SEED, min(step, n - lo), float($DEPTH), first=lo, mapq=bool($MAPQ)))
    print(path, os.path.getsize(path), flush=True)
PY
cat $F > /dev/null
PATHS=${PATHS:-'"" "--host-parse"'}
eval "set -- $PATHS"
for extra in "$@"; do
  for rep in 1 2; do
    a=$(date +%s.%N)
    timeout -k 10 600 ./build/sid --stats $extra $FLAGS $F > /dev/null 2> $O/e2e_stats.txt || { echo "sid rc=$?"; cat $O/e2e_stats.txt; exit 1; }
    b=$(date +%s.%N)
    w=$(python3 -c "print('%.4f' % ($b - $a))")
    echo "{\"path\": \"${extra:-device}\", \"flags\": \"$FLAGS\", \"rep\": $rep, \"wall_s\": $w, \"sites\": $SITES, \"stats\": $(tail -1 $O/e2e_stats.txt)}" | tee -a $O/e2e.jsonl
  done
done
t0=$(date +%s.%N)
timeout -k 10 600 ./oracle/_build/sid_oracle $FLAGS $S > /dev/null || exit 1
t1=$(date +%s.%N)
python3 -c "print('{\"path\": \"oracle\", \"flags\": \"$FLAGS\", \"sites\": $SAMPLE, \"seconds\": %.3f, \"sites_per_s\": %.1f}' % ($t1-$t0, $SAMPLE/($t1-$t0)))" | tee -a $O/e2e.jsonl
