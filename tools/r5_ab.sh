#!/bin/bash
# Round 5 A/B of the product library against sdp-net_amd/lib_base (the previous build): GEMM tests,
# GEMM per M forward with the model's epilogues, M forward interleaved, epilogue stamps (new).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B=$GRAFT_REPO_ROOT/sdp-net_amd/lib_base/libsdpnet_hip.so
step() {  # name limit cmd...
  local n=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$n.log" 2>&1
  local rc=$?
  echo "== $n rc=$rc"; tail -3 "gpurun_out/$n.log"
  if [ $rc -ne 0 ]; then echo "ABORT after $n"; exit $rc; fi
}
step r5ab_tests 600 python -u -m pytest tests/test_gpu_kernels.py -k "gemm" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
for v in base new base new; do
  if [ $v = base ]; then export SDPNET_HIP_LIB=$B; else unset SDPNET_HIP_LIB; fi
  step r5ab_g_$v 300 python tools/gemm_bench.py --shapes mixer_cc,mixer_up,mixer_down,enc_qkv,enc_o,enc_ff1,enc_ff2
  grep -v amdgpu gpurun_out/r5ab_g_$v.log | awk '{print $1, $(NF-11), $(NF-10)}'
  step r5ab_m_$v 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary
  grep -o '"value": [0-9.]*' gpurun_out/r5ab_m_$v.log
done
unset SDPNET_HIP_LIB
SDPNET_HIP_LIB=sdp-net_amd/lib_stamps/libsdpnet_hip.so step r5ab_stamps 400 python tools/gemm_stamps.py --shapes mixer_cc,mixer_down,enc_o --epi-wait 0
grep -E "^[a-z]|epilogue|kloop|prologue" gpurun_out/r5ab_stamps.log
SDPNET_HIP_LIB=sdp-net_amd/lib_stamps/libsdpnet_hip.so step r5ab_astamps 300 python tools/attn_stamps.py
cat gpurun_out/r5ab_astamps.log | grep -v amdgpu
