#!/bin/bash
# PMC passes (instruction mix, stalls, LDS, memory) of the C2 device path for
# each build in BUILDS, to compare kernels between variants.  gpurun_out/pab_<build>/
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for v in ${BUILDS:-build build_b}; do
  export SID_LIB_PATH=$GRAFT_REPO_ROOT/$v/libsid.so
  B="python3 $GRAFT_REPO_ROOT/bench.py --device-only --steps 2 --device-steps 2"
  run() {
    local g=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/pab_$v/pmc_$g -o p -- $B > $O/pab_$v.$g.log 2>&1
  }
  run insts SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit $?
  run stall SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU SQ_WAVE_CYCLES || exit $?
  run stall2 SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES SQ_INSTS_BRANCH || echo "stall2 failed"
  python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $O/pab_$v | grep -E "sid_local_put|sid_local_len|sid_parse_kernel|sid_index_count|sid_index_emit" > $O/pab_$v.txt
  cat $O/pab_$v.txt
done
