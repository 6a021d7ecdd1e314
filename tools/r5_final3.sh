#!/bin/bash
# Round 5 closing measurement set on the final build: full GPU suite + smoke, the default bench line,
# the M forward kernel summary + traffic (kernel trace + FETCH_SIZE + WRITE_SIZE passes), attention /
# dwconv PMC.  Every GPU step has its own time limit; a crash or timeout ends the call.
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
step r5f3_tests 1500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread
step r5f3_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r5f3_bench 900 python bench.py
BP="python bench.py --config m --steps 10 --warmup 3 --no-cpu-baseline --no-secondary"
step r5f3_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r5f3_prof -o run --output-format csv -- $BP
step r5f3_pmcF 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r5f3_pmcF -o run --output-format csv -- $BP
step r5f3_pmcW 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r5f3_pmcW -o run --output-format csv -- $BP
python tools/prof_summary.py --round r05b --config m --graph --out gpurun_out/r5f3_profiles \
  --prof gpurun_out/r5f3_prof --fetch gpurun_out/r5f3_pmcF --write gpurun_out/r5f3_pmcW \
  --bench-log gpurun_out/r5f3_prof.log --cmd "bench.py --config m --steps 10 --warmup 3 --no-cpu-baseline --no-secondary" > /dev/null || exit 1
rm -rf gpurun_out/r5f3_pmcF gpurun_out/r5f3_pmcW
find gpurun_out/r5f3_prof -name "*kernel_trace.csv" -delete
step r5f3_pmc_na 400 bash tools/r5_pmc_na.sh
cat gpurun_out/r5_na_pmc.json | python -c "import json,sys; d=json.load(sys.stdin); [print(k, {kk: v for kk, v in d[k].items() if kk != 'counters'}) for k in d]"
echo ALLDONE
