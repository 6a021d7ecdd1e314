# Upper bounds on the M step from the non-GEMM kernels: skip the depthwise conv (1), attention (2),
# LN stats (4) in turn (timing only: wrong results), interleaved with the full step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1 2 4 0 1 2 4; do
  SDPNET_DEBUG_SKIP=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r4_skip_$v.log 2>&1 || { tail -20 gpurun_out/r4_skip_$v.log; exit 1; }
  echo "M skip=$v $(tail -n 1 gpurun_out/r4_skip_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
