# XL training A/B of the static-priority PH2 loops: lib = GEMM static / wgrad per-section flips,
# lib_alt = both static, lib_alt2 = both per-section flips (the previous build)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$PWD/sdp-net_amd
lib() { case $1 in d) echo $R/lib/libsdpnet_hip.so;; s) echo $R/lib_alt/libsdpnet_hip.so;; o) echo $R/lib_alt2/libsdpnet_hip.so;; esac; }
for v in o d s o d s; do
  SDPNET_HIP_LIB=$(lib $v) timeout -k 10 300 python bench.py --config xl_train --steps 20 --no-cpu-baseline > gpurun_out/r4_prio2_$v.log 2>&1 || { tail -20 gpurun_out/r4_prio2_$v.log; exit 1; }
  echo "XL train $v $(tail -n 1 gpurun_out/r4_prio2_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r4_prio2_m.log 2>&1 && echo "M d $(tail -n 1 gpurun_out/r4_prio2_m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
