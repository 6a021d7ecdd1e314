# A/B of the PH2 k-loop priority scheme: per-section s_setprio (default lib) vs static priority for
# wave group 1 (lib_alt, -DSDP_PH2_PRIO=1) vs no s_setprio (lib_alt2, -DSDP_PH2_PRIO=2)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$PWD/sdp-net_amd
lib() { case $1 in d) echo $R/lib/libsdpnet_hip.so;; s) echo $R/lib_alt/libsdpnet_hip.so;; n) echo $R/lib_alt2/libsdpnet_hip.so;; esac; }
for v in d s n; do
  SDPNET_HIP_LIB=$(lib $v) timeout -k 10 200 python tools/gemm_bench.py --shapes sq8192,mixer_down,mixer_up,mixer_cc,enc_qkv,enc_ff1 > gpurun_out/r4_prio_g_$v.log 2>&1 || { tail -20 gpurun_out/r4_prio_g_$v.log; exit 1; }
  echo "== gemm $v"; grep -v amdgpu gpurun_out/r4_prio_g_$v.log
done
for v in d s n d s n; do
  SDPNET_HIP_LIB=$(lib $v) timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r4_prio_m_$v.log 2>&1 || { tail -20 gpurun_out/r4_prio_m_$v.log; exit 1; }
  echo "M $v $(tail -n 1 gpurun_out/r4_prio_m_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
