set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_train.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/r3_train5.log 2>&1 || { tail -40 gpurun_out/r3_train5.log; exit 1; }
grep -E "passed|failed|XL-dim|PASSED|FAILED" gpurun_out/r3_train5.log | tail -30
