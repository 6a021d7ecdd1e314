set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu -k "attn or attention" > gpurun_out/r3_attn_t.log 2>&1 || { tail -30 gpurun_out/r3_attn_t.log; exit 1; }
tail -1 gpurun_out/r3_attn_t.log
for i in 1 2; do
for pc in 2 0; do
SDPNET_ATTN_PER_CU=$pc timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/r3_attnab_$pc.log 2>&1 || { tail -30 gpurun_out/r3_attnab_$pc.log; exit 1; }
echo "per_cu=$pc $(grep -o '"value": [0-9.]*' gpurun_out/r3_attnab_$pc.log)"
done
done
