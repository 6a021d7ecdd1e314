set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in 4,4 2,4 2,8; do
    log=gpurun_out/gm2_${i}_${v/,/_}.log
    SDPNET_TMP_GM=$v timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary > $log 2>&1 || { tail -5 $log; exit 1; }
    echo "m GM(small,big)=$v: $(grep -o '"value": [0-9.]*' $log | head -1)"
  done
done
