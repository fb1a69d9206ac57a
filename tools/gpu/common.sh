# shared by tools/gpu/*.sh (sourced): the repo root on the box, gpurun_out,
# TMPDIR=/tmp for rocprofv3, and `summary` for a bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=${O:-$PWD/gpurun_out}
mkdir -p "$O"
summary() {   # bench json -> one line
    python3 - "$1" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
dp = d.get("device_path", {})
print(d["config"]["workload"][:3], "value %.4g" % d["value"], "ms %.2f" % d["ms_per_step"],
      "device %.3f ms" % dp.get("ms_per_step", 0), {k: round(v, 3) for k, v in dp.get("stages_ms", {}).items()},
      "roof %.3f" % d["roofline"]["frac"], "cpu", (d.get("cpu_baseline") or {}).get("value"),
      "cli", (d.get("cli") or {}).get("wall_s"))
PY
}
