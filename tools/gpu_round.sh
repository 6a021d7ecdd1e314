#!/bin/bash
# GPU-box script: kernel tests -> model tests -> bench.  Stops at the first
# crash/timeout (exit codes other than 0/1), continues past plain test failures.
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ===" ; date
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc" >> "gpurun_out/$name.log"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name rc=$rc"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    kern) step kern 900 python -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider -rf ;;
    model) step model 1200 python -m pytest tests/test_gpu_model.py -q -p no:cacheprovider -rf ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py --steps 10 --warmup 3 ;;
    benchq) step benchq 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    gemm) step gemm 600 python tools/gemm_bench.py --streams 1 --kernels 3,5 ;;
    prof) export TMPDIR=/tmp; rm -rf gpurun_out/prof
          step prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-graph --prof-steps 1 ;;
  esac
done
