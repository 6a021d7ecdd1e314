#!/bin/bash
# Round 5: attn_fa5 (one 8-wave workgroup per CU, double-buffered K/V, producer wave) -- tests,
# kernel time against fa4, phase stamps, M forward interleaved with SDPNET_ATTN_KERNEL=4 / 6 / 7.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name limit cmd...
  local n=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$n.log" 2>&1
  local rc=$?
  echo "== $n rc=$rc"; tail -3 "gpurun_out/$n.log"
  if [ $rc -ne 0 ]; then echo "ABORT after $n"; exit $rc; fi
}
step r5f_tests 400 python -u -m pytest tests/test_gpu_kernels.py -k "attention" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step r5f_kb 200 python tools/kern_bench.py --only attn --attn-kerns 4,6,7,4,6,7
SDPNET_HIP_LIB=sdp-net_amd/lib_stamps/libsdpnet_hip.so step r5f_as7 200 python tools/attn_stamps.py --kernel 7
grep -v amdgpu gpurun_out/r5f_as7.log
for k in 4 6 7 4 6 7; do
  SDPNET_ATTN_KERNEL=$k step r5f_m_$k 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary
  grep -o '"value": [0-9.]*' gpurun_out/r5f_m_$k.log
done
