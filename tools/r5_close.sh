#!/bin/bash
# Round 5 closing check on the committed build: full GPU suite, smoke, default bench line.
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
step r5c_tests 1500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread
step r5c_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r5c_bench 900 python bench.py
echo ALLDONE
