# Depthwise weight gradient: GPU tests, the kernel alone at the XL shape, and interleaved XL
# training A/B against the library built from HEAD (sdp-net_amd/lib_base).  Repo root, GPU box.
set -e
mkdir -p gpurun_out
B=$GRAFT_REPO_ROOT/sdp-net_amd/lib_base/libsdpnet_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_kernels.py -m gpu -x -q -k "dw_wgrad" \
  --timeout 120 --timeout-method thread > gpurun_out/dwg_tests.log 2>&1 || { tail -30 gpurun_out/dwg_tests.log; exit 1; }
tail -n 1 gpurun_out/dwg_tests.log
SDPNET_HIP_LIB=$B timeout -k 10 120 python tools/dw_wgrad_bench.py 2>&1 | grep dw_wgrad | sed 's/^/base /'
timeout -k 10 120 python tools/dw_wgrad_bench.py 2>&1 | grep dw_wgrad | sed 's/^/new  /'
for rep in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export SDPNET_HIP_LIB=$B; else unset SDPNET_HIP_LIB; fi
    timeout -k 10 240 python bench.py --config xl_train --steps 40 --warmup 5 --no-cpu-baseline \
      > gpurun_out/dwg_$v.log 2>&1 || { tail -20 gpurun_out/dwg_$v.log; exit 1; }
    echo "$v $(tail -n 1 gpurun_out/dwg_$v.log | grep -o '"value": [0-9.]*')"
  done
done
