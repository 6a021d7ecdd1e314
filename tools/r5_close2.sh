#!/bin/bash
# Round 5 closing check on the attn_fa6 build: full GPU suite, smoke, default bench line, and the
# XL forward kernel summary + traffic (kernel trace, FETCH_SIZE and WRITE_SIZE passes, short runs).
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
step r5d_tests 1500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread
step r5d_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r5d_bench 900 python bench.py
BP="python bench.py --config xl --steps 5 --warmup 2 --no-cpu-baseline --no-secondary"
step r5d_prof_xl 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r5d_prof_xl -o run --output-format csv -- $BP
step r5d_pmcF_xl 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r5d_pmcF_xl -o run --output-format csv -- $BP
step r5d_pmcW_xl 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r5d_pmcW_xl -o run --output-format csv -- $BP
python tools/prof_summary.py --round r05c_xl --config xl --graph --out gpurun_out/r5d_profiles \
  --prof gpurun_out/r5d_prof_xl --fetch gpurun_out/r5d_pmcF_xl --write gpurun_out/r5d_pmcW_xl \
  --bench-log gpurun_out/r5d_prof_xl.log --cmd "bench.py --config xl --steps 5 --warmup 2 --no-cpu-baseline --no-secondary" > /dev/null || exit 1
rm -rf gpurun_out/r5d_pmcF_xl gpurun_out/r5d_pmcW_xl
find gpurun_out/r5d_prof_xl -name "*kernel_trace.csv" -delete
ls gpurun_out/r5d_profiles
echo ALLDONE
