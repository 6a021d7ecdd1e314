#!/bin/bash
# Round 5: what the non-GEMM kernel families cost the M step (diagnostic library, kernel-skip masks:
# bit 0 depthwise conv, bit 1 attention, bit 2 LN statistics; results are wrong while skipping), then
# the default bench line of the product library.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SDPNET_HIP_LIB=sdp-net_amd/lib_stamps/libsdpnet_hip.so timeout -k 10 400 python tools/skip_bench.py --masks 0,1,2,3,4 > gpurun_out/r5_skip.log 2>&1 || { tail -5 gpurun_out/r5_skip.log; exit 1; }
grep -v amdgpu gpurun_out/r5_skip.log
timeout -k 10 900 python bench.py > gpurun_out/r5_bench_last.log 2>&1 || { tail -5 gpurun_out/r5_bench_last.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r5_bench_last.log | head -3
