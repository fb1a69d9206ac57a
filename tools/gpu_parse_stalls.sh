#!/bin/bash
# where the parse's time goes: wave cycles split into parked (WAIT_ANY),
# issue-stalled (WAIT_INST_ANY) and issuing (ACTIVE_INST_*), the texture
# addresser's busy cycles, L1 accesses and stalls; one pass per block group
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --device-only --steps 2 --device-steps 2"
run() {
    local g=$1; shift
    ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/stall/pmc_$g -o p -- $B > $O/stall_$g.log 2>&1 )
}
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES || exit $?
run ta TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES || exit $?
run tcp TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES || exit $?
run sq2 SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_THREAD_CYCLES_VALU SQ_CYCLES || exit $?
python3 - <<'PY'
import csv, os, glob, collections
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/stall"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
for f in glob.glob(O + "/pmc_*/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")
        k = k.replace("(anonymous namespace)::", "")[:40]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]] += 1
out = {}
for k, v in agg.items():
    if any(s in k for s in ("parse", "index", "local_put", "local_len")):
        out[k] = {c: x / max(1, cnt[k][c]) * 1.0 for c, x in v.items()}
import json
json.dump(out, open(os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/stall_summary.json", "w"), indent=1)
for k, v in out.items():
    print(k, {c: f"{x:.4g}" for c, x in sorted(v.items())})
PY
