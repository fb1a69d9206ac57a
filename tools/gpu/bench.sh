#!/bin/bash
# bench.py lines per config: gpurun_out/bench_<cfg>_<TAG>.json (+ .err), one
# summary line each.   usage: tools/gpu/bench.sh TAG C2 [C3 C4 C5] [-- extra bench args]
. "$(dirname "$0")/common.sh"
TAG=${1:-run}; shift
CFGS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do CFGS+=("$1"); shift; done
[ "$1" = "--" ] && shift
for c in "${CFGS[@]:-C2}"; do
    timeout -k 10 600 python3 -u bench.py --config $c "$@" > $O/bench_${c,,}_$TAG.json 2> $O/bench_${c,,}_$TAG.err \
        || { echo "bench $c failed"; tail $O/bench_${c,,}_$TAG.err; exit 1; }
    summary $O/bench_${c,,}_$TAG.json
done
