#!/bin/bash
# round-2 first bench pass: C2 (with extras), C3, C4, C5 on one GPU + a kernel trace of C2
set -e
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err
timeout -k 10 300 python -u bench.py --config C3 --steps 10 > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 300 python -u bench.py --config C4 --steps 2 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err
timeout -k 10 300 python -u bench.py --config C5 --steps 2 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/c2trace -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-extras > $GRAFT_REPO_ROOT/$O/c2trace.log 2>&1
