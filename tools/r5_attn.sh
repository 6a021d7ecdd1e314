#!/bin/bash
# Round 5: attention K/V staging by buffer LDS-DMA with per-lane offsets precomputed (tests, kernel
# time, model, PMC), GEMM per M forward with the model's epilogues, and epilogue sub-phase stamps.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name limit cmd...
  local n=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$n.log" 2>&1
  local rc=$?
  echo "== $n rc=$rc"; tail -4 "gpurun_out/$n.log"
  if [ $rc -ne 0 ]; then echo "ABORT after $n"; exit $rc; fi
}
step r5_at_tests 400 python -u -m pytest tests/test_gpu_kernels.py -k "attention" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step r5_at_model_tests 400 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step r5_at_kb 200 python tools/kern_bench.py --only attn --attn-kerns 3,4
step r5_at_kbxl 200 python tools/kern_bench.py --only attn --attn-kerns 3 --shape xl
for i in 1 2; do
  step r5_at_m_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary
  grep -o '"value": [0-9.]*' gpurun_out/r5_at_m_$i.log
done
step r5_at_pmc 400 bash tools/r5_pmc_na.sh
step r5_at_gemm 400 python tools/gemm_bench.py --shapes mixer_cc,mixer_up,mixer_down,enc_qkv,enc_o,enc_ff1,enc_ff2
grep "GEMM time" gpurun_out/r5_at_gemm.log
SDPNET_HIP_LIB=sdp-net_amd/lib_stamps/libsdpnet_hip.so step r5_at_stamps 400 python tools/gemm_stamps.py --shapes mixer_cc,mixer_down,enc_o,mixer_up --epi-wait 0
grep -E "^[a-z]|epilogue|kloop|prologue" gpurun_out/r5_at_stamps.log
