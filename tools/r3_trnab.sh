set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_kernels.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu -k "dw_wgrad" > gpurun_out/r3_ab0.log 2>&1 || { tail -40 gpurun_out/r3_ab0.log; exit 1; }
tail -1 gpurun_out/r3_ab0.log
for i in 1 2; do
for f in 1 0; do
SDPNET_TRAIN_FUSED_EPI=$f timeout -k 10 300 python -u bench.py --config xl_train --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3_ab_$f.log 2>&1 || { tail -30 gpurun_out/r3_ab_$f.log; exit 1; }
echo "fused=$f $(grep -o '"value": [0-9.]*' gpurun_out/r3_ab_$f.log)"
done
done
rm -rf gpurun_out/tprof2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/tprof2 -o run --output-format csv -- python bench.py --config xl_train --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/tprof2.log 2>&1 || { tail -20 gpurun_out/tprof2.log; exit 1; }
echo done
