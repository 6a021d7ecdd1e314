set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_train_kernels.py -k "wgrad" > gpurun_out/r4_train_tests.log 2>&1 || { tail -30 gpurun_out/r4_train_tests.log; exit 1; }
tail -1 gpurun_out/r4_train_tests.log
for k in 4 2 4 2; do
  SDPNET_GEMM_KLOOP_PHASES=$k timeout -k 10 300 python bench.py --config xl_train --steps 20 --no-cpu-baseline > gpurun_out/r4_train_$k.log 2>&1 || { tail -20 gpurun_out/r4_train_$k.log; exit 1; }
  echo "xl_train kloop=$k $(tail -n 1 gpurun_out/r4_train_$k.log | cut -c1-230)"
done
rm -rf gpurun_out/r4_tprof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_tprof -o run --output-format csv -- python bench.py --config xl_train --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r4_tprof.log 2>&1 || { tail -20 gpurun_out/r4_tprof.log; exit 1; }
python tools/stats_table.py gpurun_out/r4_tprof 2>/dev/null | head -40 || true
