#!/bin/bash
# Round 5: dwconv3 addressing rewrite (tests, kernel time, model) + GEMM epilogue sub-phase stamps
# (diagnostic library) for the residual / non-residual shapes.
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
step r5_epi_tests 300 python -u -m pytest tests/test_gpu_kernels.py -k "dwconv" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step r5_epi_kb 200 python tools/kern_bench.py --only dw
for i in 1 2; do
  step r5_epi_m_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary
  grep -o '"value": [0-9.]*' gpurun_out/r5_epi_m_$i.log
done
SDPNET_HIP_LIB=sdp-net_amd/lib_stamps/libsdpnet_hip.so step r5_epi_stamps 400 python tools/gemm_stamps.py --shapes mixer_cc,mixer_cc_nores,mixer_down,enc_qkv,mixer_up --epi-wait 0,1
cat gpurun_out/r5_epi_stamps.log
