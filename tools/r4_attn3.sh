set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_train_kernels.py tests/test_gpu_train_modules.py > gpurun_out/r4_attn3_tests.log 2>&1 || { tail -30 gpurun_out/r4_attn3_tests.log; exit 1; }
tail -1 gpurun_out/r4_attn3_tests.log
timeout -k 10 200 python tools/attn_train_bench.py > gpurun_out/r4_attn3_bench.log 2>&1 || { tail -20 gpurun_out/r4_attn3_bench.log; exit 1; }
grep -v amdgpu gpurun_out/r4_attn3_bench.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --config xl_train --steps 20 --no-cpu-baseline > gpurun_out/r4_attn3_xlt_$i.log 2>&1 || { tail -20 gpurun_out/r4_attn3_xlt_$i.log; exit 1; }
  echo "xl_train $(tail -n 1 gpurun_out/r4_attn3_xlt_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
