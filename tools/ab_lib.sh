set -o pipefail
B=$GRAFT_REPO_ROOT/sdp-net_amd/lib_base/libsdpnet_hip.so
for v in base new base new; do
  if [ $v = base ]; then export SDPNET_HIP_LIB=$B; else unset SDPNET_HIP_LIB; fi
  timeout -k 10 200 python tools/gemm_bench.py --shapes sq8192,mixer_down,mixer_up,mixer_cc,enc_qkv > gpurun_out/ab_g_$v.log 2>&1 || exit 1
  echo "== $v"; grep -v amdgpu gpurun_out/ab_g_$v.log | awk '{print $1, $(NF-11), $(NF-10)}'
  timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ab_b_$v.log 2>&1 || exit 1
  grep -o '"value": [0-9.]*' gpurun_out/ab_b_$v.log
done
