#!/bin/bash
# Round 6 closing check: full GPU suite + smoke, then the default bench line (traffic tied to this build).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/r6_tests.sh || exit 1
timeout -k 10 800 python bench.py > gpurun_out/r6_final_bench.log 2>&1 || { tail -5 gpurun_out/r6_final_bench.log; exit 1; }
grep '^{' gpurun_out/r6_final_bench.log | tail -1 | cut -c1-300
