#!/bin/bash
# Round 5 A/B against sdp-net_amd/lib_base (the HEAD build): software-pipelined LN backward rows --
# LN / training kernel tests, LN-backward microbenchmark, XL training step interleaved.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B=$GRAFT_REPO_ROOT/sdp-net_amd/lib_base/libsdpnet_hip.so
step() {  # name limit cmd...
  local n=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$n.log" 2>&1
  local rc=$?
  echo "== $n rc=$rc"; tail -2 "gpurun_out/$n.log"
  if [ $rc -ne 0 ]; then echo "ABORT after $n"; exit $rc; fi
}
step r5e_tests 600 python -u -m pytest tests/test_gpu_train_kernels.py tests/test_train.py tests/test_gpu_train_modules.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider
for v in base new base new; do
  if [ $v = base ]; then export SDPNET_HIP_LIB=$B; else unset SDPNET_HIP_LIB; fi
  step r5e_lnb_$v 120 python tools/lnb_bench.py
  step r5e_xlt_$v 400 python bench.py --config xl_train --steps 20 --warmup 3 --no-cpu-baseline --no-secondary
  grep -o '"value": [0-9.]*' gpurun_out/r5e_xlt_$v.log
done
