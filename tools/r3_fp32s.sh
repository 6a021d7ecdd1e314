set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_train_modules.py tests/test_train.py tests/test_compile.py tests/test_gpu_train_kernels.py tests/test_gpu_model.py -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/r3_fp32s.log 2>&1 || { tail -60 gpurun_out/r3_fp32s.log; exit 1; }
grep -E "bf16|fp32|ratio|passed|failed" gpurun_out/r3_fp32s.log | tail -30
timeout -k 10 300 python -u bench.py --config xl_train --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3_xlt32.log 2>&1 || { tail -30 gpurun_out/r3_xlt32.log; exit 1; }
grep '"metric"' gpurun_out/r3_xlt32.log | cut -c1-400
SDPNET_TRAIN_FP32_STREAM=0 timeout -k 10 300 python -u bench.py --config xl_train --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3_xlt16.log 2>&1 || { tail -30 gpurun_out/r3_xlt16.log; exit 1; }
grep '"metric"' gpurun_out/r3_xlt16.log | cut -c1-400
