set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in 0 1 3; do
    log=gpurun_out/apc_${i}_$v.log
    SDPNET_ATTN_PER_CU=$v timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary > $log 2>&1 || { tail -5 $log; exit 1; }
    echo "m ATTN_PER_CU=$v: $(grep -o '"value": [0-9.]*' $log | head -1)"
  done
done
