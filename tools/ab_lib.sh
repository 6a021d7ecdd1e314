#!/bin/bash
# Interleaved same-box A/B on one GPU box (one gpurun call).
#   tools/ab_lib.sh [--knob VAR=a,b] [--tests "PYTEST ARGS"] WHAT...
# Without --knob: the product library (sdp-net_amd/lib) against sdp-net_amd/lib_base/libsdpnet_hip.so
# (build that one from the commit to compare against and copy it there).  With --knob: the product
# library with VAR=a against VAR=b (an SDPNET_* switch; bench.py records it in config.knobs).
# WHAT (each run as A, B, A, B): m (M forward), xl (XL forward), xlt (XL bs120 training step),
# gemm (single-stream GEMM per M forward, tools/gemm_bench.py), attn / attnxl / dw (tools/kern_bench.py),
# lnb (LN backward microbenchmark).  Logs: gpurun_out/ab_<what>_<variant>_<i>.log.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
KNOB="" TESTS=""
while [ $# -gt 0 ]; do
  case $1 in
    --knob) KNOB=$2; shift 2 ;;
    --tests) TESTS=$2; shift 2 ;;
    *) break ;;
  esac
done
step() {  # name limit cmd...
  local n=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$n.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "== $n rc=$rc"; tail -5 "gpurun_out/$n.log"; echo "ABORT after $n"; exit $rc; fi
}
if [ -n "$TESTS" ]; then
  step ab_tests 900 python -u -m pytest $TESTS -x -q --timeout 240 --timeout-method thread -p no:cacheprovider
  tail -1 gpurun_out/ab_tests.log
fi
if [ -n "$KNOB" ]; then
  VAR=${KNOB%%=*}; VALS=${KNOB#*=}; A=${VALS%%,*}; B=${VALS#*,}
  variants="$A $B $A $B"
else
  BASE=$GRAFT_REPO_ROOT/sdp-net_amd/lib_base/libsdpnet_hip.so
  [ -f "$BASE" ] || { echo "no $BASE"; exit 1; }
  variants="base new base new"
fi
i=0
for v in $variants; do
  i=$((i + 1))
  if [ -n "$KNOB" ]; then export "$VAR=$v"; elif [ $v = base ]; then export SDPNET_HIP_LIB=$BASE; else unset SDPNET_HIP_LIB; fi
  for what in "$@"; do
    n=ab_${what}_${v}_$i
    case $what in
      m) step $n 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary ;;
      xl) step $n 400 python bench.py --config xl --steps 20 --warmup 3 --no-cpu-baseline --no-secondary ;;
      xlt) step $n 400 python bench.py --config xl_train --steps 20 --warmup 3 --no-cpu-baseline --no-secondary ;;
      gemm) step $n 400 python tools/gemm_bench.py --shapes mixer_cc,mixer_up,mixer_down,enc_qkv,enc_o,enc_ff1,enc_ff2 ;;
      attn) step $n 200 python tools/kern_bench.py --only attn --attn-kerns 4,6 ;;
      attnxl) step $n 200 python tools/kern_bench.py --only attn --attn-kerns 3 --shape xl ;;
      dw) step $n 200 python tools/kern_bench.py --only dw ;;
      lnb) step $n 120 python tools/lnb_bench.py ;;
      *) echo "unknown WHAT $what"; exit 2 ;;
    esac
    echo "$what $v: $(grep -ho '"value": [0-9.]*\|GEMM time per M forward[^:]*: [0-9.]* ms\|^attention k[0-9].*us \|^dwconv_ln k[0-9].*us \|ln_bwd.*us ' gpurun_out/$n.log | tr '\n' ' ')"
  done
done
