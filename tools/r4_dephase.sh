# Round 4 experiment: does de-phasing the tile rounds shorten the GEMM epilogue / prologue?
# (stamps library; first-round workgroups wait ((b >> 3) & 3) * D ticks), plus the 1- vs 2-stream split.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/gemm_bench.py --schedules 0 --streams 1,2 --reps 20 \
  --shapes mixer_cc,mixer_up,mixer_down,enc_qkv,enc_o,enc_ff1,enc_ff2 > gpurun_out/r4_streams.log 2>&1 || { tail -20 gpurun_out/r4_streams.log; exit 1; }
grep -v amdgpu gpurun_out/r4_streams.log | cut -c1-150
timeout -k 10 300 python tools/gemm_stamps.py --schedules 0 --dephase 0,400,800 \
  --shapes mixer_cc,enc_qkv,mixer_down > gpurun_out/r4_dephase.log 2>&1 || { tail -20 gpurun_out/r4_dephase.log; exit 1; }
grep -v "in-epilogue" gpurun_out/r4_dephase.log
