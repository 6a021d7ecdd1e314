set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in -1 4 8; do
    log=gpurun_out/tgm_${i}_$v.log
    SDPNET_GEMM_GROUP_M=$v timeout -k 10 400 python bench.py --config xl_train --steps 15 --warmup 3 --no-cpu-baseline --no-secondary > $log 2>&1 || { tail -5 $log; exit 1; }
    echo "xlt GROUP_M=$v: $(grep -o '"value": [0-9.]*' $log | head -1)"
  done
done
