set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in 1 0; do
    log=gpurun_out/xcd_${i}_$v.log
    SDPNET_TMP_XCD=$v timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary > $log 2>&1 || { tail -5 $log; exit 1; }
    echo "m XCD_MAP=$v: $(grep -o '"value": [0-9.]*' $log | head -1)"
  done
done
