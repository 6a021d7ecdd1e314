#!/bin/bash
# Full GPU suite + smoke (one gpurun call).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/r6_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r6_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r6_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_smoke.log 2>&1 || { tail -20 gpurun_out/r6_smoke.log; exit 1; }
tail -1 gpurun_out/r6_smoke.log
