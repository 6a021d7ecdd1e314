"""Summarise tools/gemm_pmc.sh: per GEMM shape of tools/gemm_bench.py (dispatch order, 3 warm-up
+ N timed launches per shape), the kernel time (kernel trace), effective clock
(GRBM_GUI_ACTIVE / 8 XCDs / wall, MI355X guide 'DVFS give-back'), MFMA busy share, wait /
issue breakdown, LDS bank conflicts and HBM-side traffic (2*FETCH_SIZE + WRITE_SIZE, KiB units,
gfx950 correction) against the algorithmic bytes.

  python tools/gemm_pmc_summary.py gpurun_out/gpmc [--json out.json]
"""
import csv
import os
import json
import sys
from collections import defaultdict

SHAPES = [("mixer_cc", 50176, 768, 768, False, True), ("mixer_up", 50176, 3072, 768, False, False),
          ("mixer_down", 50176, 768, 3072, False, True), ("enc_qkv", 51200, 2304, 768, False, False),
          ("enc_o", 51200, 768, 768, False, True), ("enc_ff1", 51200, 3072, 768, True, False),
          ("enc_ff2", 51200, 768, 3072, True, True)]
WARM = 3
NCU, PEAK = 256, 2516.6e12


def gemm_rows(path):
    kname = os.environ.get("PMC_KERNEL", "gemm_bf16_8ph")
    return [r for r in csv.DictReader(open(path)) if kname in r["Kernel_Name"]]


def blocks(rows):
    """Consecutive dispatches of one (kernel, grid) = one shape of gemm_bench (run in SHAPES order);
    the first WARM of each block are dropped."""
    rows = sorted(rows, key=lambda r: int(r["Dispatch_Id"]))
    out, key = [], None
    for r in rows:
        k = (r["Kernel_Name"], r.get("Grid_Size", r.get("Grid_Size_X", "")))
        if k != key:
            out.append([])
            key = k
        out[-1].append(r)
    return [b[WARM:] if len(b) > WARM else b for b in out]


def main():
    d = sys.argv[1]
    bl = blocks(gemm_rows(f"{d}/trace/run_kernel_trace.csv"))
    if len(bl) != len(SHAPES):
        raise SystemExit(f"expected {len(SHAPES)} shape blocks in the kernel trace, found {len(bl)}")
    dur = {s: [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 for r in b] for s, b in enumerate(bl)}
    ctr = defaultdict(lambda: defaultdict(list))
    for p in "ABFWH":
        try:
            rows = gemm_rows(f"{d}/{p}/run_counter_collection.csv")
        except FileNotFoundError:
            continue
        # counter rows: one per (dispatch, counter); group dispatches into shape blocks the same way
        disp = {}
        for r in rows:
            disp.setdefault(int(r["Dispatch_Id"]), []).append(r)
        order = sorted(disp)
        seq = [disp[i][0] for i in order]
        bks = blocks(seq)
        if len(bks) != len(SHAPES):
            print(f"pass {p}: {len(bks)} shape blocks, skipped")
            continue
        for s, b in enumerate(bks):
            for r0 in b:
                for r in disp[int(r0["Dispatch_Id"])]:
                    ctr[s][r["Counter_Name"]].append((float(r["Counter_Value"]),
                                                       (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9))
    out = []
    hdr = ("shape", "us", "TF/s", "%pk", "clk GHz", "%pk@clk", "MFMA busy", "wait", "issue-stall", "active",
           "LDS cf/act", "HBM MB", "alg MB", "x alg", "L2 hit")
    print("  ".join(f"{h:>10s}" for h in hdr))
    for s, (name, M, N, K, b, r) in enumerate(SHAPES):
        t = sum(dur[s]) / len(dur[s])
        fl = 2.0 * M * N * K
        c = {k: sum(v for v, _ in lst) / len(lst) for k, lst in ctr[s].items()}
        walls = {k: sum(w for _, w in lst) / len(lst) for k, lst in ctr[s].items()}
        clk = c.get("GRBM_GUI_ACTIVE", 0) / 8 / walls.get("GRBM_GUI_ACTIVE", 1) / 1e9
        # MFMA pipe busy: SQ_VALU_MFMA_BUSY_CYCLES summed over the SIMDs of all CUs vs the
        # available SIMD cycles (GRBM_GUI_ACTIVE / 8 per XCD clock x 1024 SIMDs)
        simd_cycles = c.get("GRBM_GUI_ACTIVE", 0) / 8 * NCU * 4
        mbusy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / simd_cycles if simd_cycles else 0
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        alg = 2 * (M * K + N * K + M * N * (2 if r else 1)) + (4 * N if b else 0)
        hbm = (2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024
        hit = c.get("TCC_HIT_sum", 0) / max(1.0, c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0))
        rec = dict(shape=name, M=M, N=N, K=K, us=round(t * 1e6, 1), tflops=round(fl / t / 1e12, 1),
                   frac=round(fl / t / PEAK, 4), eff_clock_ghz=round(clk, 3),
                   frac_at_clock=round(fl / t / (PEAK * clk / 2.4), 4) if clk else None,
                   mfma_busy=round(mbusy, 4), sq_wait_any=round(c.get("SQ_WAIT_ANY", 0) / wc, 3),
                   sq_wait_inst_any=round(c.get("SQ_WAIT_INST_ANY", 0) / wc, 3),
                   sq_active_inst_any=round(c.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3),
                   lds_conflict_per_active=round(c.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, c.get("SQ_LDS_IDX_ACTIVE", 1)), 4),
                   hbm_bytes=int(hbm), algorithmic_bytes=alg, hbm_over_alg=round(hbm / alg, 3),
                   l2_hit=round(hit, 3), raw=c)
        out.append(rec)
        print("  ".join(f"{v:>10}" for v in (name, rec["us"], rec["tflops"], f"{100 * rec['frac']:.1f}",
                                             rec["eff_clock_ghz"], f"{100 * (rec['frac_at_clock'] or 0):.1f}",
                                             f"{100 * mbusy:.1f}", rec["sq_wait_any"], rec["sq_wait_inst_any"],
                                             rec["sq_active_inst_any"], rec["lds_conflict_per_active"],
                                             round(hbm / 1e6, 1), round(alg / 1e6, 1), rec["hbm_over_alg"],
                                             rec["l2_hit"])))
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
