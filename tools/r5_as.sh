set -o pipefail
mkdir -p gpurun_out
for k in 6 4; do
SDPNET_HIP_LIB=sdp-net_amd/lib_stamps/libsdpnet_hip.so timeout -k 10 200 python tools/attn_stamps.py --kernel $k > gpurun_out/r5_as_$k.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/r5_as_$k.log
done
