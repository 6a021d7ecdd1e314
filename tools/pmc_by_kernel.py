"""Per-kernel mean of rocprofv3 --pmc counter values (one counter_collection.csv per pass).

  python tools/pmc_by_kernel.py DIR1 [DIR2 ...] --match dwconv3,attn_fa4 [--json out.json]

For every kernel whose name contains one of the --match substrings: dispatch count, mean kernel
duration and the mean per-dispatch value of every counter found in the passes, plus derived ratios
(LDS-active share of wave cycles, VALU / LDS / MFMA instructions per wave, effective clock).
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    args = [a for a in sys.argv[1:]]
    match = args[args.index("--match") + 1].split(",") if "--match" in args else [""]
    js = args[args.index("--json") + 1] if "--json" in args else None
    dirs = [a for i, a in enumerate(args) if not a.startswith("--") and (i == 0 or not args[i - 1].startswith("--"))]
    per = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(dict)
    for d in dirs:
        try:
            rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
        except FileNotFoundError:
            print(f"{d}: no counter_collection.csv")
            continue
        for r in rows:
            name = r["Kernel_Name"]
            key = next((m for m in match if m in name), None)
            if key is None:
                continue
            per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[key][(d, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {}
    for k, c in per.items():
        m = {n: sum(v) / len(v) for n, v in c.items()}
        t = sum(dur[k].values()) / max(1, len(dur[k]))
        waves = m.get("SQ_WAVES", 0) or 1
        wc = m.get("SQ_WAVE_CYCLES", 0) or 1
        rec = dict(dispatches=len(dur[k]), mean_us=round(t * 1e6, 2), counters=m)
        rec["valu_per_wave"] = round(m.get("SQ_INSTS_VALU", 0) / waves, 1)
        rec["lds_per_wave"] = round(m.get("SQ_INSTS_LDS", 0) / waves, 1)
        rec["mfma_per_wave"] = round(m.get("SQ_INSTS_MFMA", 0) / waves, 1)
        rec["wait_any_frac"] = round(m.get("SQ_WAIT_ANY", 0) / wc, 3)
        rec["wait_inst_any_frac"] = round(m.get("SQ_WAIT_INST_ANY", 0) / wc, 3)
        if "GRBM_GUI_ACTIVE" in m and t:
            rec["clock_ghz"] = round(m["GRBM_GUI_ACTIVE"] / 8 / t / 1e9, 3)
            busy = m["GRBM_GUI_ACTIVE"] / 8 * 256  # CU cycles
            if "SQ_LDS_IDX_ACTIVE" in m:
                rec["lds_idx_active_per_cu_cycle"] = round(m["SQ_LDS_IDX_ACTIVE"] / busy, 3)
            if "SQ_LDS_BANK_CONFLICT" in m and "SQ_LDS_IDX_ACTIVE" in m:
                rec["lds_conflict_share"] = round(m["SQ_LDS_BANK_CONFLICT"] / max(1, m["SQ_LDS_IDX_ACTIVE"]), 3)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                rec["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (busy * 4), 3)
        out[k] = rec
        print(k, json.dumps({a: b for a, b in rec.items() if a != "counters"}))
    if js:
        json.dump(out, open(js, "w"), indent=1)


if __name__ == "__main__":
    main()
