set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_kernels.py -k "specialised or kloop or attention or patchify" > gpurun_out/r4_spec2_tests.log 2>&1 || { tail -30 gpurun_out/r4_spec2_tests.log; exit 1; }
tail -1 gpurun_out/r4_spec2_tests.log
timeout -k 10 400 $T tests/test_gpu_train_modules.py tests/test_train.py -k "patcher or embedding_activation or compile" > gpurun_out/r4_spec2_tests2.log 2>&1 || { tail -30 gpurun_out/r4_spec2_tests2.log; exit 1; }
tail -1 gpurun_out/r4_spec2_tests2.log
timeout -k 10 200 python tools/kern_bench.py --only attn --shape m > gpurun_out/r4_fs_kb_m.log 2>&1 || { tail -20 gpurun_out/r4_fs_kb_m.log; exit 1; }
grep attention gpurun_out/r4_fs_kb_m.log
timeout -k 10 200 python tools/kern_bench.py --only attn --shape xl --attn-kerns 3,5 > gpurun_out/r4_fs_kb_xl.log 2>&1 || { tail -20 gpurun_out/r4_fs_kb_xl.log; exit 1; }
grep attention gpurun_out/r4_fs_kb_xl.log
for k in 0 1 0 1; do
  SDPNET_GEMM_EPI_SPEC=$k timeout -k 10 300 python bench.py --config xl_train --steps 20 --no-cpu-baseline > gpurun_out/r4_spec2_t_$k.log 2>&1 || { tail -20 gpurun_out/r4_spec2_t_$k.log; exit 1; }
  echo "xl_train spec=$k $(tail -n 1 gpurun_out/r4_spec2_t_$k.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
for k in 4 5 4 5; do
  SDPNET_ATTN_KERNEL=$k timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r4_fs_m_$k.log 2>&1 || { tail -20 gpurun_out/r4_fs_m_$k.log; exit 1; }
  echo "M attn=$k $(tail -n 1 gpurun_out/r4_fs_m_$k.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
for k in 3 5 3 5; do
  SDPNET_ATTN_KERNEL=$k timeout -k 10 300 python bench.py --config xl --no-cpu-baseline > gpurun_out/r4_fs_xl_$k.log 2>&1 || { tail -20 gpurun_out/r4_fs_xl_$k.log; exit 1; }
  echo "XL attn=$k $(tail -n 1 gpurun_out/r4_fs_xl_$k.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
