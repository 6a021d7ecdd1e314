set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_kernels.py -k "kloop" > gpurun_out/r4_diag_tests.log 2>&1 || { tail -30 gpurun_out/r4_diag_tests.log; exit 1; }
tail -1 gpurun_out/r4_diag_tests.log
timeout -k 10 200 python tools/gemm_phases.py --shapes mixer_cc,enc_ff1,sq8192 > gpurun_out/r4_diag_phases.log 2>&1 || { tail -20 gpurun_out/r4_diag_phases.log; exit 1; }
grep -E "mean|clock|^[a-z]" gpurun_out/r4_diag_phases.log
timeout -k 10 200 python tools/gemm_stamps.py --shapes mixer_cc,enc_ff1,mixer_down --schedules 0 > gpurun_out/r4_diag_stamps.log 2>&1 || { tail -20 gpurun_out/r4_diag_stamps.log; exit 1; }
grep -v amdgpu gpurun_out/r4_diag_stamps.log
