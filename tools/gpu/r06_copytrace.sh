#!/bin/bash
# the C2 value leg's copies and kernels on one timeline: rocprofv3 kernel and
# memory-copy traces (no counters) over a short bench run -> gpurun_out/copytrace_r06/
. "$(dirname "$0")/common.sh"
P=$O/copytrace_r06
mkdir -p $P
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace ${CT_EXTRA:-} --output-format csv -d $P -o ct -- \
      python3 $OLDPWD/bench.py --steps 5 --warmup 2 --no-cpu > $P/bench.json 2> $P/bench.log ) \
    || { echo "copy trace failed"; tail -3 $P/bench.log; exit 1; }
ls $P
