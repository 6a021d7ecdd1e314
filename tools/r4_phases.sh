set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/gemm_phases.py --shapes mixer_down,enc_qkv,mixer_cc > gpurun_out/r4_phases.log 2>&1 || { tail -20 gpurun_out/r4_phases.log; exit 1; }
grep -v amdgpu gpurun_out/r4_phases.log
