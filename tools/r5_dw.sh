#!/bin/bash
# Round 5: depthwise-conv tier 4 (DPP-moved tap rows) -- tests, kernel timing, model A/B against
# tier 3, then PMC passes over dwconv3 / attn_fa4.
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
step r5_dw_tests 300 python -u -m pytest tests/test_gpu_kernels.py -k "dwconv" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step r5_dw_kb 200 python tools/kern_bench.py --only dw,attn --attn-kerns 4
for k in 3 4 3 4; do
  SDPNET_DW_KERNEL=$k step r5_dw_m_$k 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary
  grep -o '"value": [0-9.]*' gpurun_out/r5_dw_m_$k.log
done
step r5_pmc_na 400 bash tools/r5_pmc_na.sh
cat gpurun_out/r5_na_pmc.json | head -60
