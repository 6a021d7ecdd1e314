#!/bin/bash
# Round 6: XL bs120 training step timeline (rocprofv3 kernel trace -> tools/train_trace.py)
set -o pipefail
mkdir -p gpurun_out/ttrace
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/ttrace -o run --output-format csv -- \
  python3 bench.py --config xl_train --steps 3 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/ttrace.log 2>&1 \
  || { tail -20 gpurun_out/ttrace.log; exit 1; }
f=$(ls gpurun_out/ttrace/*/run_kernel_trace.csv gpurun_out/ttrace/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/train_trace.py "$f" ${FAM:-seg_colsum_v4} gpurun_out/r6_xltrain_launches.csv > gpurun_out/r6_xltrain_timeline.txt 2>&1
rm -rf gpurun_out/ttrace
cat gpurun_out/r6_xltrain_timeline.txt
