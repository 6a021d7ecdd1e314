# Round 4: training-kernel tests touched this round, then a kernel trace of the benchmarked
# command (graph replay, 2 sub-batch streams) -> overlap analysis, plus GEMM traffic PMC passes.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_kernels.py -x -q --timeout 300 --timeout-method thread -k "ce_loss or attn or softmax" > gpurun_out/r4_trk.log 2>&1 || { tail -30 gpurun_out/r4_trk.log; exit 1; }
tail -n 1 gpurun_out/r4_trk.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_modules.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_trm.log 2>&1 || { tail -30 gpurun_out/r4_trm.log; exit 1; }
tail -n 1 gpurun_out/r4_trm.log
timeout -k 10 900 python -u -m pytest tests/test_compile.py -x -q --timeout 600 --timeout-method thread -m gpu -k ddp > gpurun_out/r4_compile.log 2>&1 || { tail -40 gpurun_out/r4_compile.log; exit 1; }
tail -n 1 gpurun_out/r4_compile.log
O=gpurun_out/r4t; rm -rf $O; mkdir -p $O
CMD="bench.py --steps 20 --warmup 3 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python $CMD > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
tail -n 1 $O/trace.log | cut -c1-300
python tools/trace_overlap.py $O/trace/run_kernel_trace.csv > $O/overlap.txt 2>&1; cat $O/overlap.txt
CMD="bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/F -o run --output-format csv -- python $CMD > $O/F.log 2>&1 || { tail -20 $O/F.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/W -o run --output-format csv -- python $CMD > $O/W.log 2>&1 || { tail -20 $O/W.log; exit 1; }
ls $O/F $O/W
