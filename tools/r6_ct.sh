#!/bin/bash
# Round 6: cross-tile GEMM correctness + solo timing (one gpurun call).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "cross_tile" -p no:cacheprovider > gpurun_out/r6_ct_test.log 2>&1 || { tail -30 gpurun_out/r6_ct_test.log; exit 1; }
tail -2 gpurun_out/r6_ct_test.log
timeout -k 10 500 python tools/gemm_bench.py --shapes mixer_cc,mixer_up,mixer_down,enc_qkv,enc_o,enc_ff1,enc_ff2 \
  --ct ${CTS:-0,1:2:4096,1:1:4096,2:2:4096,3:2:4096} > gpurun_out/r6_ct_bench.log 2>&1 || { tail -20 gpurun_out/r6_ct_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6_ct_bench.log
