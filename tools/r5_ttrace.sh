#!/bin/bash
# XL bs120 training step kernel trace (per-queue timeline, tools/train_trace.py).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/r5_ttrace
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/r5_ttrace -o run --output-format csv -- python bench.py --config xl_train --steps 3 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/r5_ttrace.log 2>&1 || exit 1
python tools/train_trace.py gpurun_out/r5_ttrace/run_kernel_trace.csv seg_colsum_v4 > gpurun_out/r5_ttrace.txt || exit 1; cat gpurun_out/r5_ttrace.txt
rm -f gpurun_out/r5_ttrace/run_kernel_trace.csv
