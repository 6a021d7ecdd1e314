# A/B of the fa4 softmax chunk size (ATTN_CH 4 vs 7) via an alternate library (sdp-net_amd/lib_alt)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ALT=$PWD/sdp-net_amd/lib_alt/libsdpnet_hip.so
DEF=$PWD/sdp-net_amd/lib/libsdpnet_hip.so
SDPNET_HIP_LIB=$ALT timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "attention" > gpurun_out/r4_ch_tests.log 2>&1 || { tail -30 gpurun_out/r4_ch_tests.log; exit 1; }
tail -1 gpurun_out/r4_ch_tests.log
timeout -k 10 200 python tools/kern_bench.py --only attn --attn-kerns 4 > gpurun_out/r4_ch_kb4.log 2>&1 && grep attention gpurun_out/r4_ch_kb4.log
SDPNET_HIP_LIB=$ALT timeout -k 10 200 python tools/kern_bench.py --only attn --attn-kerns 4 > gpurun_out/r4_ch_kb7.log 2>&1 && grep attention gpurun_out/r4_ch_kb7.log
for v in 4 7 4 7; do
  if [ $v = 7 ]; then L=$ALT; else L=$DEF; fi
  SDPNET_HIP_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r4_ch_m_$v.log 2>&1 || { tail -20 gpurun_out/r4_ch_m_$v.log; exit 1; }
  echo "M CH=$v $(tail -n 1 gpurun_out/r4_ch_m_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
