set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
SDPNET_GEMM_KLOOP_PHASES=2 timeout -k 10 400 $T tests/test_gpu_kernels.py tests/test_gpu_train_kernels.py -k "gemm or wgrad" > gpurun_out/r4_ph2_tests.log 2>&1 || { tail -30 gpurun_out/r4_ph2_tests.log; exit 1; }
tail -2 gpurun_out/r4_ph2_tests.log
timeout -k 10 300 python tools/gemm_bench.py --schedules 0 --kloop 4,2 > gpurun_out/r4_ph2_gemm.log 2>&1 || { tail -20 gpurun_out/r4_ph2_gemm.log; exit 1; }
grep "per M forward" gpurun_out/r4_ph2_gemm.log
for k in 4 2 4 2; do
  SDPNET_GEMM_KLOOP_PHASES=$k timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r4_ph2_bench_$k.log 2>&1 || { tail -20 gpurun_out/r4_ph2_bench_$k.log; exit 1; }
  echo "m kloop=$k $(tail -n 1 gpurun_out/r4_ph2_bench_$k.log | cut -c1-200)"
done
for k in 4 2 4 2; do
  SDPNET_GEMM_KLOOP_PHASES=$k timeout -k 10 300 python bench.py --config xl_train --steps 20 --no-cpu-baseline > gpurun_out/r4_ph2_xlt_$k.log 2>&1 || { tail -20 gpurun_out/r4_ph2_xlt_$k.log; exit 1; }
  echo "xl_train kloop=$k $(tail -n 1 gpurun_out/r4_ph2_xlt_$k.log | cut -c1-200)"
done
SDPNET_GEMM_KLOOP_PHASES=2 timeout -k 10 200 python tools/gemm_phases.py --shapes mixer_down,mixer_cc > gpurun_out/r4_ph2_phases.log 2>&1 || { tail -20 gpurun_out/r4_ph2_phases.log; exit 1; }
grep -v amdgpu gpurun_out/r4_ph2_phases.log | tail -22
