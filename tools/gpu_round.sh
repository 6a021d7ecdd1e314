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
    all) step all 1500 python -u -m pytest tests/ -m gpu -q -p no:cacheprovider -rf --timeout 240 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py --steps 10 --warmup 3 ;;
    benchq) step benchq 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    streams) step s1 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --streams 1 &&
             step s2 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --streams 2 &&
             step s3 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --streams 3 &&
             step s4 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --streams 4 ;;
    kb) step kb 300 python tools/kern_bench.py ;;
    pmc) export TMPDIR=/tmp; rm -rf gpurun_out/pmc*
         step pmc1 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES -d gpurun_out/pmc1 -o run --output-format csv -- python tools/kern_bench.py --reps 3 &&
         step pmc2 600 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmc2 -o run --output-format csv -- python tools/kern_bench.py --reps 3 &&
         step pmc3 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc3 -o run --output-format csv -- python tools/kern_bench.py --reps 3 &&
         step pmc4 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc4 -o run --output-format csv -- python tools/kern_bench.py --reps 3 ;;
    gpmc) export TMPDIR=/tmp; rm -rf gpurun_out/gpmc*
         GB="python tools/gemm_bench.py --reps 2 --kernels 14 --shapes mixer_up,mixer_down,sq8192"
         step gpmcA 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS -d gpurun_out/gpmcA -o run --output-format csv -- $GB &&
         step gpmcB 600 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE SQ_INSTS_VMEM -d gpurun_out/gpmcB -o run --output-format csv -- $GB &&
         step gpmcC 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/gpmcC -o run --output-format csv -- $GB &&
         step gpmcD 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/gpmcD -o run --output-format csv -- $GB ;;
    prof) export TMPDIR=/tmp; rm -rf gpurun_out/prof gpurun_out/pmcF gpurun_out/pmcW
          BP="python bench.py --steps 3 --warmup 1 --no-graph --streams 1 --no-cpu-baseline --prof-steps 1"
          step prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- $BP &&
          step pmcF 900 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcF -o run --output-format csv -- $BP &&
          step pmcW 900 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcW -o run --output-format csv -- $BP ;;
  esac
done
