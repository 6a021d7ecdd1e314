set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_kernels.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu -k "train_epilogues or act_fwd or flash" > gpurun_out/r3_te1.log 2>&1 || { tail -40 gpurun_out/r3_te1.log; exit 1; }
tail -1 gpurun_out/r3_te1.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_train_modules.py tests/test_train.py tests/test_compile.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/r3_te2.log 2>&1 || { tail -40 gpurun_out/r3_te2.log; exit 1; }
tail -1 gpurun_out/r3_te2.log
timeout -k 10 300 python -u bench.py --config xl_train --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3_te_b32.log 2>&1 || { tail -30 gpurun_out/r3_te_b32.log; exit 1; }
grep -o '"value": [0-9.]*, "unit[^,]*, "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/r3_te_b32.log
SDPNET_TRAIN_FP32_STREAM=0 timeout -k 10 300 python -u bench.py --config xl_train --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3_te_b16.log 2>&1 || { tail -30 gpurun_out/r3_te_b16.log; exit 1; }
grep -o '"value": [0-9.]*, "unit[^,]*, "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/r3_te_b16.log
