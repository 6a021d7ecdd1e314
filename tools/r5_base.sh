#!/bin/bash
# Round 5 baseline GPU call: full GPU suite, the default bench line, GEMM PMC passes (MFMA busy,
# clock, traffic) and a kernel-trace profile of the headline bench.  Every GPU step has its own
# time limit; a crash / timeout ends the call.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name limit cmd...
  local n=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$n.log" 2>&1
  local rc=$?
  echo "== $n rc=$rc"; tail -3 "gpurun_out/$n.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $n"; exit $rc; fi
  return $rc
}
step r5b_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1
step r5b_bench 400 python bench.py --steps 20 --warmup 5 || exit 1
step r5b_gpmc 900 bash tools/gemm_pmc.sh gpurun_out/r5b_gpmc || exit 1
python tools/gemm_pmc_summary.py gpurun_out/r5b_gpmc --json gpurun_out/r5b_gemm_pmc.json > gpurun_out/r5b_gemm_pmc.md 2>&1; tail -15 gpurun_out/r5b_gemm_pmc.md
step r5b_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r5b_prof -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary || exit 1
ls gpurun_out/r5b_prof/*
