# Round-end validation on the GPU box (repo root): every GPU test, smoke(), the default bench line,
# the XL training bench line and a kernel trace of the XL training step.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_gputest.log 2>&1 || { tail -30 gpurun_out/final_gputest.log; exit 1; }
tail -n 1 gpurun_out/final_gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -n 1 gpurun_out/final_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/final_bench.log 2>&1 || { tail -20 gpurun_out/final_bench.log; exit 1; }
tail -n 1 gpurun_out/final_bench.log | cut -c1-200
timeout -k 10 300 python bench.py --config xl_train --no-cpu-baseline > gpurun_out/final_xlt.log 2>&1 || { tail -20 gpurun_out/final_xlt.log; exit 1; }
tail -n 1 gpurun_out/final_xlt.log | cut -c1-200
rm -rf gpurun_out/prof_xlt2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_xlt2 -o run --output-format csv -- python bench.py --config xl_train --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_xlt2.log 2>&1 || { tail -20 gpurun_out/prof_xlt2.log; exit 1; }
python tools/stats_table.py gpurun_out/prof_xlt2/run_kernel_stats.csv --steps-seen 5 --title "XL bs120 training step" > gpurun_out/prof_xlt2_table.md 2>&1 || true
