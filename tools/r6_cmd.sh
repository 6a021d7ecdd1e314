set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary --no-graph > gpurun_out/evb_0.log 2>&1 && echo "fused, no graph: $(grep -o '"value": [0-9.]*' gpurun_out/evb_0.log | head -1)"
SDPNET_EVAL_FP32_STREAM=1 timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary --no-graph > gpurun_out/evb_1.log 2>&1 && echo "fp32 stream, no graph: $(grep -o '"value": [0-9.]*' gpurun_out/evb_1.log | head -1)"
tail -3 gpurun_out/evb_1.log | cut -c1-300
