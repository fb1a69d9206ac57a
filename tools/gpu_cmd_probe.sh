set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/engine_probe.py --runs 3 --modes device,host,pinned > gpurun_out/probe1.log 2>&1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run -- python3 $GRAFT_REPO_ROOT/tools/engine_probe.py --runs 2 --modes device > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1
