# XL training A/B over SDPNET_WGRAD_CUS (workgroups the split-K dW grid aims for), interleaved.
# Repo root, GPU box.
set -e
mkdir -p gpurun_out
for rep in 1 2 3; do
  for cus in ${WGCUS_LIST:-256 384 512}; do
    SDPNET_WGRAD_CUS=$cus timeout -k 10 240 python bench.py --config xl_train --steps 40 --warmup 5 \
      --no-cpu-baseline > gpurun_out/wgcus_$cus.log 2>&1 || { tail -20 gpurun_out/wgcus_$cus.log; exit 1; }
    echo "cus=$cus $(tail -n 1 gpurun_out/wgcus_$cus.log | grep -o '"value": [0-9.]*')"
  done
done
