#!/bin/bash
# Round 6: M forward with the cross-tile GEMM on the N = 768 shapes vs without (interleaved, one box).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "cross_tile" -p no:cacheprovider > gpurun_out/r6_ct_test.log 2>&1 || { tail -30 gpurun_out/r6_ct_test.log; exit 1; }
tail -1 gpurun_out/r6_ct_test.log
for i in 1 2 3; do
  for v in off ${CTV:--1,2,768,768}; do
    if [ $v = off ]; then unset SDPNET_GEMM_CT; else export SDPNET_GEMM_CT=$v; fi
    timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/r6_ctab_${i}_$v.log 2>&1 || { tail -5 gpurun_out/r6_ctab_${i}_$v.log; exit 1; }
    echo "$v: $(grep -o '"value": [0-9.]*' gpurun_out/r6_ctab_${i}_$v.log)"
  done
done
