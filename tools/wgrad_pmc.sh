#!/bin/bash
# PMC passes over the weight-gradient microbenchmark (tools/dw_bench.py, XL bs120 shapes, the
# 8-phase gemm_wgrad_8ph kernel), one pass per counter group, summarised like the forward GEMM.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/wpmc}
rm -rf "$OUT"; mkdir -p "$OUT"
GB="python tools/dw_bench.py --reps 4 --impl 8ph"
run() {  # name counters...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d "$OUT/$n" -o run --output-format csv -- $GB > "$OUT/$n.log" 2>&1 || { echo "pass $n failed"; tail -5 "$OUT/$n.log"; exit 1; }
}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- $GB > "$OUT/trace.log" 2>&1 || exit 1
run A SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT
run B SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES
run F FETCH_SIZE
run W WRITE_SIZE
run H TCC_HIT_sum TCC_MISS_sum
PMC_KERNEL=gemm_wgrad_8ph python tools/gemm_pmc_summary.py "$OUT" --json "$OUT.json" > "$OUT.md" 2>&1; cat "$OUT.md"
grep -h "8ph" "$OUT/trace.log" | head -8
rm -rf "$OUT"
echo done
