# GEMM HBM traffic of the benchmarked command (graph + 2 sub-batch streams): kernel trace and two
# separate PMC passes (FETCH_SIZE, WRITE_SIZE), then tools/prof_summary.py -> profiles/r03t_*.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/p3; rm -rf $O; mkdir -p $O
CMD="bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python $CMD > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/F -o run --output-format csv -- python $CMD > $O/F.log 2>&1 || { tail -20 $O/F.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/W -o run --output-format csv -- python $CMD > $O/W.log 2>&1 || { tail -20 $O/W.log; exit 1; }
echo done
