#!/bin/bash
# A/B of builds on the C2 value leg (pinned host text -> CSV in pinned host
# memory), interleaved on one box: gpurun_out/abv_<TAG>.log
# usage: BUILDS="build_base build" tools/gpu/ab_value.sh TAG [bench args]
# (an entry "dir@VAR=V@VAR2=W" runs dir's library with those variables set)
. "$(dirname "$0")/common.sh"
TAG=${1:-run}; shift
for r in $(seq ${REPS:-3}); do
  for v in ${BUILDS:-build_base build}; do
    IFS=@ read -r -a vv <<< "$v"
    env SID_LIB_PATH=$PWD/${vv[0]}/libsid.so "${vv[@]:1}" timeout -k 10 300 python3 -u bench.py --no-cpu --steps 20 "$@" \
        > $O/abv.json 2> $O/abv.err || { echo "$v failed"; tail -5 $O/abv.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/abv.json')); p=d['pcie']
print('$v', 'ms=%.2f' % d['ms_per_step'], 'value=%.4g' % d['value'], 'ingest=%.2f' % (p['ingest_s']*1e3), 'h2d=%.2f' % (p['h2d_s_last_step']*1e3), 'gap=%.2f' % ((p['ingest_s']-p['h2d_s_last_step'])*1e3))" | tee -a $O/abv_$TAG.log
  done
done
