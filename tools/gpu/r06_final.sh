#!/bin/bash
# round 6: the GPU suite and smoke, then the 2-rank rehearsal lines (C2, C3)
. "$(dirname "$0")/common.sh"
TAG=${1:-r06}
tools/gpu/suite.sh $TAG || exit 1
for c in C2 C3; do
  timeout -k 10 600 python3 -u bench.py --gpus 2 --allow-shared-gpu --config $c --sites 20000000 --steps 3 --warmup 1 \
      > $O/bench_rehearsal_2rank_${c,,}_$TAG.json 2> $O/bench_rehearsal_2rank_${c,,}_$TAG.err \
      || { echo "rehearsal $c failed"; tail $O/bench_rehearsal_2rank_${c,,}_$TAG.err; exit 1; }
  summary $O/bench_rehearsal_2rank_${c,,}_$TAG.json
done
exit 0
