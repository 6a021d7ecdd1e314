#!/bin/bash
# Round 6 measurement set on the current build: the default bench line, the M and XL forward kernel
# summaries + GEMM traffic (kernel trace, FETCH_SIZE and WRITE_SIZE passes of the same command), the
# GEMM per-shape PMC summary.  Every GPU step has its own time limit; a failure ends the call.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r06}
step() {  # name limit cmd...
  local n=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$n.log" 2>&1
  local rc=$?
  echo "== $n rc=$rc"; tail -2 "gpurun_out/$n.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "ABORT after $n"; exit $rc; fi
}
[ -n "$NOBENCH" ] || step ${R}_bench 900 python bench.py
for cfg in m xl; do
  if [ $cfg = m ]; then BP="python bench.py --config m --steps 10 --warmup 3 --no-cpu-baseline --no-secondary"; tag=$R
  else BP="python bench.py --config xl --steps 5 --warmup 2 --no-cpu-baseline --no-secondary"; tag=${R}_xl; fi
  rm -rf gpurun_out/${tag}_prof gpurun_out/${tag}_pmcF gpurun_out/${tag}_pmcW
  step ${tag}_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- $BP
  step ${tag}_pmcF 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${tag}_pmcF -o run --output-format csv -- $BP
  step ${tag}_pmcW 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${tag}_pmcW -o run --output-format csv -- $BP
  python tools/prof_summary.py --round $tag --config $cfg --graph --out gpurun_out/${R}_profiles \
    --prof gpurun_out/${tag}_prof --fetch gpurun_out/${tag}_pmcF --write gpurun_out/${tag}_pmcW \
    --bench-log gpurun_out/${tag}_prof.log --cmd "${BP#python }" > /dev/null || exit 1
  rm -rf gpurun_out/${tag}_pmcF gpurun_out/${tag}_pmcW
  find gpurun_out/${tag}_prof -name "*kernel_trace.csv" -delete
done
[ -n "$NOGPMC" ] || step ${R}_gpmc 1200 bash tools/gemm_pmc.sh gpurun_out/${R}_gemm_pmc
echo ALLDONE
