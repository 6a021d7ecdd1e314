set -o pipefail
mkdir -p gpurun_out
SDPNET_DW_DB=1 timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 240 --timeout-method thread -k "dwconv or mixer or conv" -p no:cacheprovider > gpurun_out/t_dwdb.log 2>&1 || { tail -30 gpurun_out/t_dwdb.log; exit 1; }
echo "DB tests: $(tail -1 gpurun_out/t_dwdb.log)"
for v in 0 1 0 1; do SDPNET_DW_DB=$v timeout -k 10 300 python3 tools/kern_bench.py --only dw > gpurun_out/kb_dw$v.log 2>&1 && echo "DB=$v $(grep -v amdgpu gpurun_out/kb_dw$v.log | tr '\n' ' ')"; done
KNOB=SDPNET_DW_DB A=0 B=1 WHAT="m" PAIRS=3 bash tools/r6_knob_ab.sh
