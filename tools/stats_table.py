"""Turn a rocprofv3 ``--kernel-trace --stats`` kernel_stats.csv into a markdown table with
per-step milliseconds (the profiled command ran ``--steps`` timed + ``--warmup`` steps, so every
kernel's total is divided by the number of steps the profiler saw).

Usage: python tools/stats_table.py STATS_CSV --steps-seen N [--title T] [--top K] > out.md
"""
import argparse
import csv
import re


def short(name: str) -> str:
    name = re.sub(r"^void ", "", name)
    name = name.split("(")[0]
    return name.replace("|", "/")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps-seen", type=int, required=True)
    ap.add_argument("--title", default="kernel stats")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    agg = {}
    for r in rows:
        k = short(r["Name"])
        c, t = agg.get(k, (0, 0))
        agg[k] = (c + int(r["Calls"]), t + int(r["TotalDurationNs"]))
    total = sum(t for _, t in agg.values())
    print(f"# {a.title}\n")
    if a.note:
        print(a.note + "\n")
    print(f"Kernel time over {a.steps_seen} profiled steps: {total / 1e6:.2f} ms "
          f"({total / 1e6 / a.steps_seen:.2f} ms per step, kernels back to back).\n")
    print("| kernel | calls/step | ms/step | % | avg µs |")
    print("|---|---|---|---|---|")
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"| `{k}` | {c / a.steps_seen:.1f} | {t / 1e6 / a.steps_seen:.2f} | {100 * t / total:.1f} | "
              f"{t / 1e3 / c:.1f} |")
    rest = sorted(agg.items(), key=lambda kv: -kv[1][1])[a.top:]
    if rest:
        t = sum(v[1] for _, v in rest)
        print(f"| ({len(rest)} others) | | {t / 1e6 / a.steps_seen:.2f} | {100 * t / total:.1f} | |")


if __name__ == "__main__":
    main()
