#!/bin/bash
# PMC A/B of the data-parallel vs stream-K schedule of the 8-phase GEMM on one shape.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/skpmc}
SHAPE=${SHAPE:-mixer_up}
rm -rf "$OUT"; mkdir -p "$OUT"
GB="python tools/gemm_bench.py --reps 3 --shapes $SHAPE --schedules 0,1"
run() {
  local n=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" -d "$OUT/$n" -o run --output-format csv -- $GB > "$OUT/$n.log" 2>&1 || { echo "pass $n failed"; tail -5 "$OUT/$n.log"; exit 1; }
}
run F FETCH_SIZE
run W WRITE_SIZE
run H TCC_HIT_sum TCC_MISS_sum
run A SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE
python tools/sk_pmc_summary.py "$OUT"
