set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/gemm_phases.py --shapes mixer_down,enc_qkv,mixer_cc > gpurun_out/r4_phases.log 2>&1 || { tail -20 gpurun_out/r4_phases.log; exit 1; }
grep -v amdgpu gpurun_out/r4_phases.log
timeout -k 10 300 python tools/skip_bench.py > gpurun_out/r4_skip.log 2>&1 || { tail -20 gpurun_out/r4_skip.log; exit 1; }
grep -v amdgpu gpurun_out/r4_skip.log | tail -6
timeout -k 10 300 python bench.py --config xl --steps 20 > gpurun_out/r4_xl.log 2>&1 || { tail -20 gpurun_out/r4_xl.log; exit 1; }
tail -n 1 gpurun_out/r4_xl.log | cut -c1-400
