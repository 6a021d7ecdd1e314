set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/tprof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/tprof -o run --output-format csv -- python bench.py --config xl_train --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/tprof.log 2>&1 || { tail -20 gpurun_out/tprof.log; exit 1; }
python tools/stats_table.py gpurun_out/tprof 2>/dev/null | head -40 || true
