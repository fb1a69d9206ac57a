#!/bin/bash
# round 6 profiles: rocprofv3 kernel traces and PMC passes (tools/gpu/profile.sh)
# for each config given: gpurun_out/prof_r06_<cfg>/
. "$(dirname "$0")/common.sh"
for c in "$@"; do
  PASSES=${PASSES:-"trace dtrace insts fetch write stall"} tools/gpu/profile.sh r06_${c,,} --config $c || exit 1
done
exit 0
