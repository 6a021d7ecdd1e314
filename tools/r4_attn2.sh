set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_train_kernels.py -k "attention" > gpurun_out/r4_attn2_tests.log 2>&1 || { tail -30 gpurun_out/r4_attn2_tests.log; exit 1; }
tail -1 gpurun_out/r4_attn2_tests.log
timeout -k 10 200 python tools/attn_train_bench.py > gpurun_out/r4_attn2_bench.log 2>&1 || { tail -20 gpurun_out/r4_attn2_bench.log; exit 1; }
grep -v amdgpu gpurun_out/r4_attn2_bench.log
rm -rf gpurun_out/r4_attn2_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_attn2_prof -o attn --output-format csv -- python tools/attn_train_bench.py --reps 10 --p 0.2 > gpurun_out/r4_attn2_prof.log 2>&1 || { tail -20 gpurun_out/r4_attn2_prof.log; exit 1; }
cut -d, -f1-5 gpurun_out/r4_attn2_prof/attn_kernel_stats.csv | cut -c1-160
