#!/bin/bash
# Round 5: PMC passes over attn_fa6 at the XL shape (bs 512, N = 260, 8 x 96), one rocprofv3 run
# per pass (SQ counters x2, FETCH_SIZE, WRITE_SIZE), summarised per kernel; raw CSVs deleted afterwards.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
KB="python tools/kern_bench.py --shape xl --only attn --attn-kerns 3 --reps 5"
O=gpurun_out/r5_xa
rm -rf $O; mkdir -p $O
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctr -d $O/p$i -o run --output-format csv -- $KB > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python tools/pmc_by_kernel.py $O/p1 $O/p2 $O/p3 $O/p4 --match attn_fa6 --json gpurun_out/r5_xa_pmc.json
rm -rf $O/p1 $O/p2 $O/p3 $O/p4
cat gpurun_out/r5_xa_pmc.json
