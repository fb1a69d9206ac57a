#!/bin/bash
# One gpurun call: CLI sanity (system HIP 7.2 runtime), smoke (torch-first
# runtime), GPU parity tests, a short bench.  Each GPU step has its own time
# limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
STEPS=${STEPS:-"cli smoke tests bench"}
for s in $STEPS; do
  case $s in
    cli)
      python3 -c "import sys; sys.path.insert(0,'.'); import sid_amd; open('$O/c1.plp','wb').write(sid_amd.synth_text(1, 10000, 30.0))" &&
      timeout -k 10 120 ./build/sid $O/c1.plp > $O/c1_local.csv 2> $O/cli.err
      rc=$?; echo "cli rc=$rc" | tee -a $O/steps.log; [ $rc -eq 0 ] || exit $rc
      ./oracle/_build/sid_oracle $O/c1.plp > $O/c1_local_oracle.csv
      cmp $O/c1_local.csv $O/c1_local_oracle.csv > $O/cli.cmp 2>&1; echo "cli cmp=$?" | tee -a $O/steps.log ;;
    smoke)
      timeout -k 10 600 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc" | tee -a $O/steps.log; [ $rc -eq 0 ] || exit $rc ;;
    tests)
      timeout -k 10 1200 python3 -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1
      rc=$?; echo "tests rc=$rc" | tee -a $O/steps.log; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 900 python3 bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err
      rc=$?; echo "bench rc=$rc" | tee -a $O/steps.log; [ $rc -eq 0 ] || exit $rc ;;
    bench_c3)
      timeout -k 10 900 python3 bench.py --method likelihood_ratio ${BENCH3_ARGS} > $O/bench_c3.json 2> $O/bench_c3.err
      rc=$?; echo "bench_c3 rc=$rc" | tee -a $O/steps.log; [ $rc -eq 0 ] || exit $rc ;;
    bench_bayes)
      timeout -k 10 900 python3 bench.py --method bayes ${BENCH3_ARGS} > $O/bench_bayes.json 2> $O/bench_bayes.err
      rc=$?; echo "bench_bayes rc=$rc" | tee -a $O/steps.log; [ $rc -eq 0 ] || exit $rc ;;
  esac
done
