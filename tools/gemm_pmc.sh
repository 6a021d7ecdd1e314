#!/bin/bash
# PMC passes over the GEMM microbenchmark at the SdP-Net-M shapes (one pass per counter
# group, as the MI355X guide prescribes), then tools/gemm_pmc_summary.py.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/gpmc}
rm -rf "$OUT"; mkdir -p "$OUT"
GB="python tools/gemm_bench.py --reps 4 --warm-s 0.05 --shapes mixer_cc,mixer_up,mixer_down,enc_qkv,enc_o,enc_ff1,enc_ff2"
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
python tools/gemm_pmc_summary.py "$OUT" --json "$OUT.json" > "$OUT.md" 2>&1; cat "$OUT.md"
rm -rf "$OUT"   # raw CSVs stay on the box (gpurun_out is capped at 64 MiB)
echo done
