set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 500 $T tests/test_gpu_train_kernels.py tests/test_train.py -k "colsum or wgrad or deterministic or side_stream" > gpurun_out/r4_colsum_tests.log 2>&1 || { tail -30 gpurun_out/r4_colsum_tests.log; exit 1; }
tail -1 gpurun_out/r4_colsum_tests.log
for k in 0 1 0 1; do
  SDPNET_COLSUM_WIDE=$k timeout -k 10 300 python bench.py --config xl_train --steps 20 --no-cpu-baseline > gpurun_out/r4_colsum_t_$k.log 2>&1 || { tail -20 gpurun_out/r4_colsum_t_$k.log; exit 1; }
  echo "xl_train wide=$k $(tail -n 1 gpurun_out/r4_colsum_t_$k.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
