set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in 256 128 64 256 128 64; do
  SDPNET_WGRAD_WGS=$w timeout -k 10 300 python bench.py --config xl_train --steps 20 --no-cpu-baseline > gpurun_out/r4_wgs_$w.log 2>&1 || { tail -20 gpurun_out/r4_wgs_$w.log; exit 1; }
  echo "wgs=$w $(tail -n 1 gpurun_out/r4_wgs_$w.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
