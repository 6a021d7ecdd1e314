# XL training A/B over stream priorities, interleaved: default, side stream high priority, training
# loop on a high-priority stream (side stream default).  Run from the repo root on the GPU box.
set -e
mkdir -p gpurun_out
: > gpurun_out/prio.txt
timeout -k 10 60 python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())" | tee -a gpurun_out/prio.txt
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --config xl_train --steps 40 --warmup 5 --no-cpu-baseline \
    > gpurun_out/prio_$name.log 2>&1 || { tail -20 gpurun_out/prio_$name.log; exit 1; }
  echo "$name $(tail -n 1 gpurun_out/prio_$name.log | grep -o '"value": [0-9.]*')" | tee -a gpurun_out/prio.txt
}
for rep in 1 2; do
  run base SDPNET_NONE=1
  run side_hi SDPNET_SIDE_PRIO=-1
  run main_hi SDPNET_BENCH_PRIO_STREAM=1
done
