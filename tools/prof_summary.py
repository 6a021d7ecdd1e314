"""Summarise one round's rocprofv3 runs of bench.py into profiles/.

  python tools/prof_summary.py --round r01 --prof gpurun_out/prof --fetch gpurun_out/pmcF \
      --write gpurun_out/pmcW --bench-log gpurun_out/prof.log

Inputs (all from the same command, `bench.py --steps 3 --warmup 1 --no-graph --streams 1
--no-cpu-baseline --prof-steps 1`, so every pass runs the same launch mix):
  --prof   rocprofv3 --kernel-trace --stats directory (run_kernel_stats.csv, run_kernel_trace.csv)
  --fetch  rocprofv3 --pmc FETCH_SIZE directory   (own pass; FETCH_SIZE costs 3 TCC slots)
  --write  rocprofv3 --pmc WRITE_SIZE directory   (own pass)
  --bench-log  stdout of the --kernel-trace run (bench.py's JSON line)

Writes profiles/<round>_kernel_stats.csv (the rocprof summary, verbatim),
profiles/<round>_summary.md and profiles/<round>_gemm_traffic.json (read by bench.py).
HBM bytes per dispatch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE/WRITE_SIZE are
KiB, and on gfx950 FETCH_SIZE counts half the bytes of 16-B-per-lane streaming reads
(MI355X_MICROARCH.md, HBM section).
"""
import argparse
import csv
import glob
import json
import os
import re
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def gemm_source_sha16():
    sys.path.insert(0, REPO)
    import bench as _bench  # the same hash bench.py compares against
    return _bench.gemm_source_sha16()


def short(name):
    name = re.sub(r"\(.*$", "", name)
    return name.replace("void ", "")


def family(name):
    """Group template instantiations: 'fast::gemm_bf16_8ph<1, 1>' -> 'gemm_bf16_8ph'."""
    s = short(name)
    s = re.sub(r"<.*$", "", s)
    return s.split("::")[-1]


def find(d, pat):
    hits = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return hits[0] if hits else None


def pmc_per_family(d, counter):
    f = find(d, "*counter_collection.csv") if d else None
    out = {}
    if not f:
        return out
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        fam = family(r["Kernel_Name"])
        v = out.setdefault(fam, [0.0, 0])
        v[0] += float(r["Counter_Value"])
        v[1] += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", required=True)
    ap.add_argument("--prof", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--bench-log")
    ap.add_argument("--out", default=os.path.join(REPO, "profiles"))
    ap.add_argument("--cmd", default="bench.py --steps 3 --warmup 1 --no-graph --streams 1 --no-cpu-baseline "
                                     "--prof-steps 1", help="the profiled bench.py arguments (for the summary text)")
    ap.add_argument("--graph", action="store_true", help="the profiled command replays the 2-stream HIP graph")
    ap.add_argument("--config", default="m", help="bench.py --config of the profiled command (m, xl)")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)

    stats = find(args.prof, "*kernel_stats.csv")
    trace = find(args.prof, "*kernel_trace.csv")
    shutil.copy(stats, os.path.join(args.out, f"{args.round}_kernel_stats.csv"))

    rows = list(csv.DictReader(open(stats)))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    fam = {}
    for r in rows:
        f = fam.setdefault(family(r["Name"]), [0.0, 0])
        f[0] += float(r["TotalDurationNs"])
        f[1] += int(r["Calls"])

    bench = None
    if args.bench_log and os.path.exists(args.bench_log):
        for line in open(args.bench_log):
            line = line.strip()
            if line.startswith("{") and '"metric"' in line:
                bench = json.loads(line)
    fetch = pmc_per_family(args.fetch, "FETCH_SIZE")
    write = pmc_per_family(args.write, "WRITE_SIZE")

    what = {"m": "SdP-Net-M, bs 256", "xl": "SdP-Net-XL, bs 512"}.get(args.config, args.config)
    L = [f"# {args.round}: rocprofv3 kernel summary of bench.py ({what}, bf16, 1 GPU)", ""]
    L.append("Command (kernel trace): `rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv "
             f"-- python {args.cmd}`  ")
    L.append("PMC passes: the same command under `rocprofv3 --pmc FETCH_SIZE` and, separately, `--pmc WRITE_SIZE`.  ")
    if args.graph:
        L.append("The benchmarked configuration: HIP-graph replay with 2 sub-batch streams (every GEMM launch is a "
                 "128-image half batch; the profiler serialises dispatches for the PMC passes), warmup + timed + "
                 "event-timed forwards, identical launch mix. Raw rocprof summary: "
                 f"`{args.round}_kernel_stats.csv`.")
    else:
        L.append("Un-graphed, single stream: 5 forwards (1 warmup + 3 timed + 1 event-timed pass), identical launch "
                 f"mix. Raw rocprof summary: `{args.round}_kernel_stats.csv`.")
    L.append("")
    L.append("| kernel (all instantiations) | calls | total ms | % | avg µs | HBM MB / call (PMC) |")
    L.append("|---|---|---|---|---|---|")
    for name, (ns, calls) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
        tb = ""
        if name in fetch and name in write and fetch[name][1]:
            per = (2 * fetch[name][0] + write[name][0]) * 1024 / fetch[name][1]
            tb = f"{per / 1e6:.1f}"
        L.append(f"| {name} | {calls} | {ns / 1e6:.2f} | {100 * ns / total:.1f} | {ns / calls / 1e3:.1f} | {tb} |")
    L.append(f"| **total** | | {total / 1e6:.2f} | 100 | | |")
    L.append("")

    traffic = None
    if bench:
        rf = bench["roofline"]
        kname = rf["kernel"]
        ns, calls = fam.get(kname, (0.0, 0))
        L.append(f"## Dominant kernel: `{kname}`")
        L.append("")
        L.append(f"- bench.py ({rf.get('achieved_basis', 'HIP events')}): {rf['launches_per_step']} launches "
                 f"per step, avg {rf['avg_launch_us']} µs, {rf['achieved']} TFLOP/s = {100 * rf['frac']:.1f} % of "
                 f"{rf['peak']} TFLOP/s dense bf16 MFMA peak")
        if calls:
            L.append(f"- rocprofv3 (same command, all {calls} dispatches): avg {ns / calls / 1e3:.2f} µs "
                     f"(ratio to bench events {ns / calls / 1e3 / rf['avg_launch_us']:.3f})")
        L.append(f"- algorithmic bytes per launch (X + W + residual + Y + bias): "
                 f"{rf['algorithmic_bytes_per_launch'] / 1e6:.1f} MB; algorithmic GFLOP per launch "
                 f"{rf['algorithmic_gflop_per_launch']}")
        if kname in fetch and kname in write and fetch[kname][1]:
            n = fetch[kname][1]
            per = (2 * fetch[kname][0] + write[kname][0]) * 1024 / n
            traffic = dict(kernel=kname, config=args.config, launches=n, fetch_size_kib_sum=fetch[kname][0],
                           write_size_kib_sum=write[kname][0], hbm_bytes_per_launch=int(per),
                           algorithmic_bytes_per_launch=rf["algorithmic_bytes_per_launch"],
                           method="(2*FETCH_SIZE + WRITE_SIZE)*1024 per dispatch, separate --pmc passes, "
                                  "averaged over all dispatches of the kernel in the bench command",
                           # the build this describes (bench.py reports traffic_stale against it)
                           lib_md5=bench.get("config", {}).get("lib_md5"),
                           gemm_src_sha16=gemm_source_sha16())
            L.append(f"- measured HBM-side traffic per launch: {per / 1e6:.1f} MB "
                     f"({per / rf['algorithmic_bytes_per_launch']:.2f}x algorithmic)")
        L.append("")
        L.append("Per-shape breakdown (bench.py's own measurement of the profiled run):")
        L.append("")
        L.append("| M x N x K | launches | avg µs | TFLOP/s |")
        L.append("|---|---|---|---|")
        for k, v in rf["per_shape"].items():
            L.append(f"| {k} | {v['launches']} | {v['avg_us']} | {v.get('tflops', v.get('tflops_co_running'))} |")
        L.append("")
        L.append(f"bench line of the profiled run: value {bench['value']} img/s, {bench['ms_per_step']} ms/step "
                 "(under the profiler — not the headline number).")
    if trace:
        L.append("")
        L.append(f"Per-dispatch trace kept on the box only (`{os.path.basename(trace)}`); the stats CSV is committed.")
    open(os.path.join(args.out, f"{args.round}_summary.md"), "w").write("\n".join(L) + "\n")
    if traffic:
        json.dump(traffic, open(os.path.join(args.out, f"{args.round}_gemm_traffic.json"), "w"), indent=1)
    print("\n".join(L))


if __name__ == "__main__":
    main()
