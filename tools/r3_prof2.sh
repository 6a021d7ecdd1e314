# Round-3 profiles of the benchmarked commands (run on the GPU box from the repo root):
# the headline M forward (HIP-graph replay, 2 sub-batch streams) and the XL training step.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_m gpurun_out/prof_xlt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_m -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_m.log 2>&1 || { tail -20 gpurun_out/prof_m.log; exit 1; }
python tools/trace_overlap.py gpurun_out/prof_m/run_kernel_trace.csv > gpurun_out/prof_m_overlap.txt 2>&1 || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_xlt -o run --output-format csv -- python bench.py --config xl_train --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_xlt.log 2>&1 || { tail -20 gpurun_out/prof_xlt.log; exit 1; }
python tools/stats_table.py gpurun_out/prof_xlt/run_kernel_stats.csv --steps-seen 5 --title "XL bs120 training step" > gpurun_out/prof_xlt_table.md 2>&1 || true
python tools/stats_table.py gpurun_out/prof_m/run_kernel_stats.csv --steps-seen 23 --title "M bs256 forward, graph + 2 streams" > gpurun_out/prof_m_table.md 2>&1 || true
