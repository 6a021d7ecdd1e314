#!/bin/bash
# Round 6: interleaved same-box A/B of one SDPNET_* knob on the M forward (and optionally XL).
#   KNOB=VAR A=val B=val [TESTK="pytest -k expr"] [WHAT="m xl"] [PAIRS=3] bash tools/r6_knob_ab.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TESTK" ]; then
  timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 240 --timeout-method thread -k "$TESTK" \
    -p no:cacheprovider > gpurun_out/r6_ab_test.log 2>&1 || { tail -30 gpurun_out/r6_ab_test.log; exit 1; }
  tail -1 gpurun_out/r6_ab_test.log
fi
for i in $(seq 1 ${PAIRS:-3}); do
  for v in "$A" "$B"; do
    export $KNOB="$v"
    for what in ${WHAT:-m}; do
      case $what in
        m) args="--steps 30 --warmup 5" ;;
        xl) args="--config xl --steps 20 --warmup 3" ;;
        xlt) args="--config xl_train --steps 20 --warmup 3" ;;
      esac
      log=gpurun_out/r6_ab_${what}_${i}_${v//[^A-Za-z0-9]/_}.log
      timeout -k 10 400 python bench.py $args --no-cpu-baseline --no-secondary > $log 2>&1 || { tail -5 $log; exit 1; }
      echo "$what $KNOB=$v: $(grep -o '"value": [0-9.]*' $log | head -1)"
    done
  done
done
