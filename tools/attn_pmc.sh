#!/bin/bash
# PMC passes over the attention microbenchmark (fa4 only); one rocprofv3 run per pass.
export TMPDIR=/tmp
mkdir -p gpurun_out
KB="python tools/kern_bench.py --only attn --attn-kerns 4 --reps 5"
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/apmc$i -o run --output-format csv -- $KB > gpurun_out/apmc$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/apmc$i.log; exit 1; }
done
echo done
python - <<'PY'
import csv, glob, collections
for d in sorted(glob.glob("gpurun_out/apmc[0-9]")):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    if not f:
        continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if "fa4" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(f"{k:26s} {sum(v) / len(v):.4g}")
PY
