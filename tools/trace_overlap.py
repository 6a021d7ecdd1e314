"""Overlap analysis of one graph-replayed forward from a rocprofv3 --kernel-trace CSV.

  rocprofv3 --kernel-trace -d gpurun_out/gtrace -o run --output-format csv -- \
      python bench.py --steps 5 --warmup 2 --no-cpu-baseline
  python tools/trace_overlap.py gpurun_out/gtrace/run_kernel_trace.csv

Takes the window between the last two forward starts (patchify launches on the first
queue), prints kernel time per kernel, how long 0/1/2 kernels (and GEMMs) ran at once,
and per-queue busy time / gaps.
"""
import collections
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"<.*", "", n)
    return n.split("::")[-1].strip().replace("void ", "")


def main(path):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"])
                for r in rows)
    pats = [e for e in ev if "patchify" in e[2]]
    # one forward per sub-batch stream per step, each stream's chain starting with a patchify;
    # graph replays run back to back, so the two streams' chains need not start together.  The
    # timed replays are the longest sequence on one queue: windows = its consecutive patchify
    # starts (one step each), all queues' kernels inside a window are analysed.
    byq = collections.defaultdict(list)
    for p in pats:
        byq[p[3]].append(p[0])
    q0 = max(byq, key=lambda q: len(byq[q]))
    fwd = sorted(byq[q0])
    wins = [(fwd[i], fwd[i + 1]) for i in range(len(fwd) - 1)]
    lens = sorted(b_ - a_ for a_, b_ in wins)
    med = lens[len(lens) // 2]
    typical = [w for w in wins if w[1] - w[0] <= 1.5 * med]
    a, b = typical[len(typical) // 2]
    print(f"{len(wins)} forward windows, median {med / 1e6:.2f} ms; analysing window {wins.index((a, b))}")
    win = [e for e in ev if a <= e[0] < b]
    busy = collections.Counter()
    for s, e, n, q in win:
        busy[n] += (e - s) / 1e6
    print(f"window {(b - a) / 1e6:.2f} ms, {len(win)} kernels, summed kernel time {sum(busy.values()):.2f} ms")
    for n, v in busy.most_common(10):
        print(f"  {n:24s} {v:7.2f} ms")
    pts = sorted([(s, 1, n) for s, e, n, q in win] + [(e, -1, n) for s, e, n, q in win])
    cur = g = 0
    last = a
    conc, gc = collections.Counter(), collections.Counter()
    for t, d, n in pts:
        conc[cur] += t - last
        gc[g] += t - last
        last = t
        cur += d
        if n.startswith("gemm"):
            g += d
    print("kernels running at once -> ms:", {k: round(v / 1e6, 2) for k, v in sorted(conc.items())})
    print("GEMMs running at once -> ms:", {k: round(v / 1e6, 2) for k, v in sorted(gc.items())})
    gu = sum(v for k, v in gc.items() if k > 0) / 1e6
    print(f"GEMM union {gu:.2f} ms = {100 * gu / ((b - a) / 1e6):.1f} % of the window; "
          f"idle (no kernel) {conc[0] / 1e6:.2f} ms")
    for q in sorted(set(e[3] for e in win)):
        ks = [e for e in win if e[3] == q]
        gaps = sum(max(0, ks[i + 1][0] - ks[i][1]) for i in range(len(ks) - 1)) / 1e6
        print(f"queue {q}: {len(ks)} kernels, busy {sum((e - s) for s, e, _, _ in ks) / 1e6:.2f} ms, gaps {gaps:.2f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
