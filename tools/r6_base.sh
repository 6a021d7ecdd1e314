set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/r6_base_m1.log 2>&1 && \
timeout -k 10 400 python tools/gemm_bench.py --shapes mixer_cc,mixer_up,mixer_down,enc_qkv,enc_o,enc_ff1,enc_ff2 --torch > gpurun_out/r6_base_gemm.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/r6_base_m2.log 2>&1
