set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/dw_wgrad_bench.py
rm -rf gpurun_out/dwg1 gpurun_out/dwg2
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE -d gpurun_out/dwg1 -o run --output-format csv -- python tools/dw_wgrad_bench.py > gpurun_out/dwg1.log 2>&1 || { tail -5 gpurun_out/dwg1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/dwg2 -o run --output-format csv -- python tools/dw_wgrad_bench.py > gpurun_out/dwg2.log 2>&1 || { tail -5 gpurun_out/dwg2.log; exit 1; }
python - <<'PY'
import csv, glob, collections
for d in ("gpurun_out/dwg1", "gpurun_out/dwg2"):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    if not f:
        print("no csv in", d); continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if "dw_wgrad" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(f"{k:24s} {sum(v)/len(v):.4g}  (n={len(v)})")
PY
