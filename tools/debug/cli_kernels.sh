#!/bin/bash
# Kernel trace of the CLI's device text path on 20M-site 30x text, a 20M-site
# 7-column text under -m quality, and 4M sites at 200x (measurement only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
python3 - <<'PY' || exit 1
import sys
sys.path.insert(0, ".")
import sid_amd
for path, n, depth, mq in (("/tmp/t30.plp", 20_000_000, 30.0, False), ("/tmp/tq.plp", 20_000_000, 30.0, True),
                           ("/tmp/t200.plp", 4_000_000, 200.0, False)):
    with open(path, "wb") as f:
        for lo in range(0, n, 2_000_000):
            f.write(sid_amd.synth_text(2, min(2_000_000, n - lo), depth, first=lo, mapq=mq))
PY
for t in "t30:" "tq:-m quality" "t200:"; do
  name=${t%%:*}; flags=${t#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cli_$name -o trace -- \
      ./build/sid --stats $flags /tmp/$name.plp > /dev/null 2> $O/cli_$name.log || { echo "cli $name rc=$?"; exit 1; }
  echo "cli $name ok"
done
