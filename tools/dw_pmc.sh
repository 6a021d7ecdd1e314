#!/bin/bash
# PMC passes over the depthwise-conv microbenchmark; one rocprofv3 run per pass.
export TMPDIR=/tmp
mkdir -p gpurun_out
KB="python tools/kern_bench.py --only dw --reps 5"
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/dpmc$i -o run --output-format csv -- $KB > gpurun_out/dpmc$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/dpmc$i.log; exit 1; }
done
echo done
