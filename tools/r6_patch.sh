set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "patchify" -p no:cacheprovider > gpurun_out/r6_patch_test.log 2>&1 || { tail -30 gpurun_out/r6_patch_test.log; exit 1; }
tail -1 gpurun_out/r6_patch_test.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/r6_patch_m.log 2>&1 && grep -o '"value": [0-9.]*' gpurun_out/r6_patch_m.log | head -1
