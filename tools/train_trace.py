"""Stream-level timeline of one training step from a rocprofv3 --kernel-trace CSV.

  rocprofv3 --kernel-trace -d gpurun_out/ttrace -o run --output-format csv -- \\
      python bench.py --config xl_train --steps 3 --warmup 2 --no-cpu-baseline --no-secondary
  python tools/train_trace.py gpurun_out/ttrace/run_kernel_trace.csv [family [launches.csv]]

Window: between the ends of the last two optimizer launches (adamw_k).  Prints the step's wall
time, per hardware queue the union of its kernels' intervals (busy) and the kernel families that
fill it, and how long 0 / 1 / 2+ kernels ran at once -- i.e. which queue is the critical path.
"""
import collections
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"<.*", "", n)
    return n.split("::")[-1].strip().replace("void ", "")


def union(iv):
    iv = sorted(iv)
    tot, cur = 0, None
    for a, b in iv:
        if cur is None or a > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    if cur:
        tot += cur[1] - cur[0]
    return tot


def main(path):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"])
                for r in rows)
    grid = {(int(r["Start_Timestamp"]), short(r["Kernel_Name"])):
            "x".join(r.get(k, "?") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z")) for r in rows}
    ends = [b for a, b, n, q in ev if n == "adamw_k"]
    if len(ends) < 2:
        sys.exit("need two optimizer launches in the trace")
    t0, t1 = ends[-2], ends[-1]
    win = [(max(a, t0), min(b, t1), n, q) for a, b, n, q in ev if b > t0 and a < t1]
    wall = t1 - t0
    print(f"step window {wall / 1e6:.2f} ms, {len(win)} kernels")
    byq = collections.defaultdict(list)
    for a, b, n, q in win:
        byq[q].append((a, b, n))
    for q, ks in sorted(byq.items(), key=lambda kv: -sum(b - a for a, b, _ in kv[1])):
        busy = union([(a, b) for a, b, _ in ks])
        fam = collections.Counter()
        for a, b, n in ks:
            fam[n] += b - a
        top = ", ".join(f"{n} {t / 1e6:.2f}" for n, t in fam.most_common(8))
        print(f"  queue {q}: {len(ks)} kernels, busy {busy / 1e6:.2f} ms ({100 * busy / wall:.0f} %), "
              f"kernel sum {sum(b - a for a, b, _ in ks) / 1e6:.2f} ms: {top}")
    # the main queue's kernels by family: calls, total, mean, and the spread of one family (argv[2])
    mq = max(byq, key=lambda q: sum(b - a for a, b, _ in byq[q]))
    fam = collections.defaultdict(list)
    for a, b, n in byq[mq]:
        fam[n].append(b - a)
    print(f"  queue {mq} by kernel (calls, total ms, mean us, min / median / max us):")
    for n, d in sorted(fam.items(), key=lambda kv: -sum(kv[1]))[:16]:
        d = sorted(d)
        print(f"    {n:28s} {len(d):5d} {sum(d) / 1e6:7.2f} {sum(d) / len(d) / 1e3:8.1f}   "
              f"{d[0] / 1e3:7.1f} {d[len(d) // 2] / 1e3:7.1f} {d[-1] / 1e3:7.1f}")
    if len(sys.argv) > 2:  # the slowest launches of one kernel family on the main queue, with their grids
        slow = sorted(((b - a, a, n) for a, b, n in byq[mq] if n == sys.argv[2]), reverse=True)[:12]
        for d, a, n in slow:
            print(f"    {n} {d / 1e3:7.1f} us at +{(a - t0) / 1e6:7.2f} ms, grid {grid.get((a, n), '?')}")
    if len(sys.argv) > 3:  # every launch of the step window: start (ms from the window), us, queue, kernel, grid
        with open(sys.argv[3], "w") as f:
            for a, b, n, q in win:
                f.write(f"{(a - t0) / 1e6:.4f},{(b - a) / 1e3:.1f},{q},{n},{grid.get((a, n), '?')}\n")
    # concurrency profile
    pts = sorted([(a, 1) for a, b, _, _ in win] + [(b, -1) for a, b, _, _ in win])
    lvl, last, hist = 0, t0, collections.Counter()
    for t, d in pts:
        hist[min(lvl, 3)] += t - last
        lvl += d
        last = t
    hist[min(lvl, 3)] += t1 - last
    print("  kernels running at once: " + ", ".join(f"{k}{'+' if k == 3 else ''}: {v / 1e6:.2f} ms"
                                                     for k, v in sorted(hist.items())))


if __name__ == "__main__":
    main(sys.argv[1])
