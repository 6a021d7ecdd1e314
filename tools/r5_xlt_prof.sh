#!/bin/bash
# XL bs120 training step: rocprofv3 kernel summary (5 steps: 2 warmup + 3 timed).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/r5x_prof_xlt
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r5x_prof_xlt -o run --output-format csv -- python bench.py --config xl_train --steps 3 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/r5x_prof_xlt.log 2>&1 || exit 1
find gpurun_out/r5x_prof_xlt -name "*kernel_trace.csv" -delete
grep -o '"value": [0-9.]*' gpurun_out/r5x_prof_xlt.log
