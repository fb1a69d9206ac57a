set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lynch_gpu.py -m gpu -k "edge" > gpurun_out/nm_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/nm_tests.log; exit 1; }
tail -3 gpurun_out/nm_tests.log
