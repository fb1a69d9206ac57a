#!/bin/bash
# round 6: device-path time (ab.sh) and FETCH/WRITE_SIZE per build (PMC passes
# over the device path), C2
. "$(dirname "$0")/common.sh"
TAG=${1:-r06}
REPS=${REPS:-3} tools/gpu/ab.sh ${TAG} || exit 1
for v in ${BUILDS}; do
  SID_LIB_PATH=$PWD/$v/libsid.so PASSES="fetch write" tools/gpu/profile.sh ${TAG}_$v || exit 1
done
exit 0
