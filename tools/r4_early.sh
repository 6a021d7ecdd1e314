set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 500 $T tests/test_gpu_kernels.py tests/test_gpu_train_kernels.py -k "gemm or wgrad" > gpurun_out/r4_early_tests.log 2>&1 || { tail -30 gpurun_out/r4_early_tests.log; exit 1; }
tail -1 gpurun_out/r4_early_tests.log
SDPNET_GEMM_EARLY_EPI=0 timeout -k 10 300 $T tests/test_gpu_kernels.py -k "kloop" > gpurun_out/r4_early_tests0.log 2>&1 || { tail -30 gpurun_out/r4_early_tests0.log; exit 1; }
tail -1 gpurun_out/r4_early_tests0.log
for k in 0 1 0 1; do
  SDPNET_GEMM_EARLY_EPI=$k timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r4_early_m_$k.log 2>&1 || { tail -20 gpurun_out/r4_early_m_$k.log; exit 1; }
  echo "M early=$k $(tail -n 1 gpurun_out/r4_early_m_$k.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
for k in 0 1 0 1; do
  SDPNET_GEMM_EARLY_EPI=$k timeout -k 10 300 python bench.py --config xl_train --steps 20 --no-cpu-baseline > gpurun_out/r4_early_t_$k.log 2>&1 || { tail -20 gpurun_out/r4_early_t_$k.log; exit 1; }
  echo "xl_train early=$k $(tail -n 1 gpurun_out/r4_early_t_$k.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
