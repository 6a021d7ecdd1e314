#!/bin/bash
# Round 5 measurement set, part 2: XL forward kernel summary + traffic (short runs: every PMC
# pass serialises the dispatches), XL training kernel summary, dwconv / attention PMC.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name limit cmd...
  local n=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$n.log" 2>&1
  local rc=$?
  echo "== $n rc=$rc"; tail -2 "gpurun_out/$n.log"
  if [ $rc -ne 0 ]; then echo "ABORT after $n"; exit $rc; fi
}
BP="python bench.py --config xl --steps 5 --warmup 2 --no-cpu-baseline --no-secondary"
step r5y_prof_xl 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r5y_prof_xl -o run --output-format csv -- $BP
step r5y_pmcF_xl 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r5y_pmcF_xl -o run --output-format csv -- $BP
step r5y_pmcW_xl 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r5y_pmcW_xl -o run --output-format csv -- $BP
python tools/prof_summary.py --round r05_xl --config xl --graph --out gpurun_out/r5y_profiles \
  --prof gpurun_out/r5y_prof_xl --fetch gpurun_out/r5y_pmcF_xl --write gpurun_out/r5y_pmcW_xl \
  --bench-log gpurun_out/r5y_prof_xl.log --cmd "bench.py --config xl --steps 5 --warmup 2 --no-cpu-baseline --no-secondary" > /dev/null || exit 1
rm -rf gpurun_out/r5y_pmcF_xl gpurun_out/r5y_pmcW_xl
find gpurun_out/r5y_prof_xl -name "*kernel_trace.csv" -delete
step r5y_prof_xlt 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r5y_prof_xlt -o run --output-format csv -- python bench.py --config xl_train --steps 3 --warmup 2 --no-cpu-baseline --no-secondary
find gpurun_out/r5y_prof_xlt -name "*kernel_trace.csv" -delete
step r5y_pmc_na 400 bash tools/r5_pmc_na.sh
ls gpurun_out/r5y_profiles
echo ALLDONE
