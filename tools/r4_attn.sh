set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/attn_train_bench.py > gpurun_out/r4_attn_bench.log 2>&1 || { tail -20 gpurun_out/r4_attn_bench.log; exit 1; }
grep -v amdgpu gpurun_out/r4_attn_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_attn_prof -o attn -- python tools/attn_train_bench.py --reps 10 > gpurun_out/r4_attn_prof.log 2>&1 || { tail -20 gpurun_out/r4_attn_prof.log; exit 1; }
find gpurun_out/r4_attn_prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
timeout -k 10 200 python tools/gemm_phases.py --shapes mixer_cc,sq8192 > gpurun_out/r4_diag_phases.log 2>&1 || { tail -20 gpurun_out/r4_diag_phases.log; exit 1; }
grep -E "mean|clock|^[a-z]" gpurun_out/r4_diag_phases.log
