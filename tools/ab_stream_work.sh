# Training GPU tests, then an interleaved XL training A/B of which stream a piece of off-chain
# backward work runs on (AB_A / AB_B: env assignments of the two arms).  Run from the repo root on
# the GPU box.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_train.py tests/test_gpu_train_kernels.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/aff_tests.log 2>&1 || { tail -30 gpurun_out/aff_tests.log; exit 1; }
tail -n 1 gpurun_out/aff_tests.log
: > gpurun_out/aff.txt
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --config xl_train --steps 40 --warmup 5 --no-cpu-baseline \
    > gpurun_out/aff_$name.log 2>&1 || { tail -20 gpurun_out/aff_$name.log; exit 1; }
  echo "$name $(tail -n 1 gpurun_out/aff_$name.log | grep -o '"value": [0-9.]*')" | tee -a gpurun_out/aff.txt
}
for rep in 1 2 3; do
  run A ${AB_A:-SDPNET_NONE=1}
  run B ${AB_B:-SDPNET_NONE=1}
done
