#!/bin/bash
# Round 5: GEMM A/Bs in one gpurun call -- trailing-MFMA hand-over (sdp_gemm_set_trail 0 / 4 / 8) and
# the epilogue drain with all LDS reads up front (lib vs lib_alt = the build before it).
set -o pipefail
mkdir -p gpurun_out
ALT=sdp-net_amd/lib_alt/libsdpnet_hip.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py -k "trail or kloop or specialised or partials_large" > gpurun_out/r5_trail_tests.log 2>&1 \
  || { tail -30 gpurun_out/r5_trail_tests.log; exit 1; }
tail -2 gpurun_out/r5_trail_tests.log
SDPNET_HIP_LIB=sdp-net_amd/lib_stamps/libsdpnet_hip.so timeout -k 10 200 python tools/gemm_phases.py \
  --shapes mixer_cc,mixer_down --trail 0,4,8 > gpurun_out/r5_trail_phases.log 2>&1 || { tail -20 gpurun_out/r5_trail_phases.log; exit 1; }
grep -E "trail|mean cycles|clock" gpurun_out/r5_trail_phases.log
GS=mixer_cc,mixer_up,mixer_down,enc_qkv,enc_o,enc_ff1,enc_ff2
timeout -k 10 300 python tools/gemm_bench.py --trail 0,4,8 --shapes sq8192,$GS > gpurun_out/r5_trail_gemm.log 2>&1 \
  || { tail -20 gpurun_out/r5_trail_gemm.log; exit 1; }
grep -E "GEMM time" gpurun_out/r5_trail_gemm.log
SDPNET_HIP_LIB=$ALT timeout -k 10 300 python tools/gemm_bench.py --shapes $GS > gpurun_out/r5_drain_gemm_alt.log 2>&1 \
  || { tail -20 gpurun_out/r5_drain_gemm_alt.log; exit 1; }
grep -E "GEMM time" gpurun_out/r5_drain_gemm_alt.log
for v in base 0 8 4 base 0 8 4; do
  if [ $v = base ]; then L=$ALT; T=0; else L=sdp-net_amd/lib/libsdpnet_hip.so; T=$v; fi
  SDPNET_HIP_LIB=$L SDPNET_GEMM_TRAIL=$T timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/r5_trail_m_$v.log 2>&1 \
    || { tail -20 gpurun_out/r5_trail_m_$v.log; exit 1; }
  echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/r5_trail_m_$v.log | head -1) $(grep -o '"gemm_union_ms_per_step": [0-9.]*' gpurun_out/r5_trail_m_$v.log)"
done
