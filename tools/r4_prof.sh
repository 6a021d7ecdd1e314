# Round-4 profile set: M and XL forward (benchmarked graph-replay command) kernel traces + GEMM
# traffic PMC passes, then the XL training step's kernel table.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4p_smoke.log 2>&1 || { tail -20 gpurun_out/r4p_smoke.log; exit 1; }
grep smoke: gpurun_out/r4p_smoke.log
for cfg in m xl; do
  O=gpurun_out/r4p_$cfg; rm -rf $O; mkdir -p $O
  timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  tail -n 1 $O/bench.log | cut -c1-300
  CMD="bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python $CMD > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
  CMD="bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline"
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/F -o run --output-format csv -- python $CMD > $O/F.log 2>&1 || { tail -20 $O/F.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/W -o run --output-format csv -- python $CMD > $O/W.log 2>&1 || { tail -20 $O/W.log; exit 1; }
done
O=gpurun_out/r4p_xlt; rm -rf $O; mkdir -p $O
timeout -k 10 300 python bench.py --config xl_train --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -n 1 $O/bench.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --config xl_train --steps 2 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
echo done
