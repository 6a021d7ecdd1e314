set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_full_tests.log 2>&1 || { tail -40 gpurun_out/r4_full_tests.log; exit 1; }
tail -3 gpurun_out/r4_full_tests.log
