#!/bin/bash
# Round 5 measurement set on one box: full GPU suite + smoke, the default bench line (driver form),
# fa4 / fa5 model A/B, GEMM PMC passes (MFMA busy, clock, traffic), kernel-trace + FETCH/WRITE
# profiles of the M and XL forwards and the XL training step, dwconv / attention PMC.
# Every GPU step has its own time limit; a crash or timeout ends the call.
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
step r5z_tests 1500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread
step r5z_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step r5z_bench 900 python bench.py || exit 1
for k in 4 6 4 6; do
  SDPNET_ATTN_KERNEL=$k step r5z_ab_$k 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary || exit 1
  grep -o '"value": [0-9.]*' gpurun_out/r5z_ab_$k.log
done
step r5z_kb 300 python tools/kern_bench.py --only dw,attn --attn-kerns 4,6 || exit 1
step r5z_gpmc 900 bash tools/gemm_pmc.sh gpurun_out/r5z_gpmc || exit 1
for cfg in m xl; do
  BP="python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-secondary"
  step r5z_prof_$cfg 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r5z_prof_$cfg -o run --output-format csv -- $BP || exit 1
  step r5z_pmcF_$cfg 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r5z_pmcF_$cfg -o run --output-format csv -- $BP || exit 1
  step r5z_pmcW_$cfg 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r5z_pmcW_$cfg -o run --output-format csv -- $BP || exit 1
  sfx=""; [ $cfg = xl ] && sfx="_xl"
  python tools/prof_summary.py --round r05$sfx --config $cfg --graph --out gpurun_out/r5z_profiles \
    --prof gpurun_out/r5z_prof_$cfg --fetch gpurun_out/r5z_pmcF_$cfg --write gpurun_out/r5z_pmcW_$cfg \
    --bench-log gpurun_out/r5z_prof_$cfg.log --cmd "bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-secondary" > /dev/null || exit 1
  rm -rf gpurun_out/r5z_pmcF_$cfg gpurun_out/r5z_pmcW_$cfg
  find gpurun_out/r5z_prof_$cfg -name "*kernel_trace.csv" -delete
done
step r5z_prof_xlt 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r5z_prof_xlt -o run --output-format csv -- python bench.py --config xl_train --steps 3 --warmup 2 --no-cpu-baseline --no-secondary || exit 1
find gpurun_out/r5z_prof_xlt -name "*kernel_trace.csv" -delete
step r5z_pmc_na 400 bash tools/r5_pmc_na.sh || exit 1
ls gpurun_out/r5z_profiles
echo ALLDONE
