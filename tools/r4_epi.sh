# Round 4: compile-time-flag GEMM epilogue -- correctness, per-shape A/B, stamps, model A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/dbg/epi_dbg.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "gemm" > gpurun_out/r4_epi_tests.log 2>&1 || { tail -30 gpurun_out/r4_epi_tests.log; exit 1; }
tail -n 2 gpurun_out/r4_epi_tests.log
timeout -k 10 300 python tools/gemm_bench.py --schedules 0 --epi-spec 0,1 --reps 20 \
  --shapes mixer_cc,mixer_up,mixer_down,enc_qkv,enc_o,enc_ff1,enc_ff2 > gpurun_out/r4_epi_bench.log 2>&1 || { tail -20 gpurun_out/r4_epi_bench.log; exit 1; }
grep -v amdgpu gpurun_out/r4_epi_bench.log | cut -c1-140
timeout -k 10 300 python tools/gemm_stamps.py --schedules 0 --shapes mixer_cc,mixer_up,mixer_down,enc_qkv > gpurun_out/r4_epi_stamps.log 2>&1 || { tail -20 gpurun_out/r4_epi_stamps.log; exit 1; }
grep -v "in-epilogue" gpurun_out/r4_epi_stamps.log
for v in 0 1 0 1; do
  SDPNET_GEMM_EPI_SPEC=$v timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r4_epi_b$v.log 2>&1 || { tail -20 gpurun_out/r4_epi_b$v.log; exit 1; }
  echo "spec=$v $(grep -o '"value": [0-9.]*' gpurun_out/r4_epi_b$v.log) $(grep -o '"achieved": [0-9.]*, "peak' gpurun_out/r4_epi_b$v.log) $(grep -o '"gemm_union_ms_per_step": [0-9.]*, "ms_per_step": [0-9.]*' gpurun_out/r4_epi_b$v.log)"
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_epi_model.log 2>&1 || { tail -30 gpurun_out/r4_epi_model.log; exit 1; }
tail -n 2 gpurun_out/r4_epi_model.log
