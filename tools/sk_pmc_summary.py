"""Per-kernel-variant means of the PMC passes of tools/sk_pmc.sh (data-parallel = the
gemm_bf16_8ph instantiation with SK=false, stream-K = SK=true)."""
import csv
import glob
import sys
from collections import defaultdict


def main(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{d}/*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "gemm_bf16_8ph" not in k:
                continue
            var = "stream-K" if ("Lb1E" in k or ", true>" in k) else "data-parallel"
            acc[var][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for var, dd in acc.items():
        per = defaultdict(list)
        for (disp, name), vals in dd.items():
            per[name].append(sum(vals))
        print(var)
        for name in sorted(per):
            v = per[name]
            print(f"  {name:26s} n={len(v):5d} mean {sum(v) / len(v):.4g}")


if __name__ == "__main__":
    main(sys.argv[1])
