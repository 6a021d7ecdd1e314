set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_train.py -x -q --timeout 120 --timeout-method thread -k "gemm or stream_k or adamw" -p no:cacheprovider > gpurun_out/r3_tests4.log 2>&1 || { tail -40 gpurun_out/r3_tests4.log; exit 1; }
tail -2 gpurun_out/r3_tests4.log
timeout -k 10 300 python tools/gemm_stamps.py --shapes mixer_cc,mixer_up,mixer_down --schedules 0 > gpurun_out/r3_stamps4.log 2>&1 || { tail -30 gpurun_out/r3_stamps4.log; exit 1; }
grep -v "amdgpu\|in-epilogue" gpurun_out/r3_stamps4.log
timeout -k 10 300 python tools/gemm_bench.py --schedules 0 --shapes mixer_cc,mixer_up,mixer_down,enc_qkv,enc_o,enc_ff1,enc_ff2 > gpurun_out/r3_gemm_ab4.log 2>&1 || { tail -30 gpurun_out/r3_gemm_ab4.log; exit 1; }
grep -v amdgpu gpurun_out/r3_gemm_ab4.log | awk '{print $1, $5, $6, $10, $11, $12, $13}'
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r3_bench4.log 2>&1 || { tail -30 gpurun_out/r3_bench4.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3_bench4.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], {k: d['roofline'][k] for k in ('achieved','frac','gemm_union_ms_per_step','per_launch_tflops','launches_per_step','avg_launch_us')})"
