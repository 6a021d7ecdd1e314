set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_kernels.py tests/test_train.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu -k "flash or gradients_match or xl_arch or dropout" > gpurun_out/r3_flash2.log 2>&1 || { tail -30 gpurun_out/r3_flash2.log; exit 1; }
tail -1 gpurun_out/r3_flash2.log
rm -rf gpurun_out/gtrace
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/gtrace -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/gtrace.log 2>&1 || { tail -20 gpurun_out/gtrace.log; exit 1; }
python tools/trace_overlap.py gpurun_out/gtrace/run_kernel_trace.csv
