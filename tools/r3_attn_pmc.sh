# One PMC pass over the XL training step: per-kernel SQ counters (what bounds the flash-attention
# backward kernels).  Own pass, SQ / GRBM counters only.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/apmc; rm -rf $O; mkdir -p $O
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA -d $O/A -o run --output-format csv -- python bench.py --config xl_train --steps 2 --warmup 1 --no-cpu-baseline > $O/A.log 2>&1 || { tail -20 $O/A.log; exit 1; }
echo done
