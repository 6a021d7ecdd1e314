"""L2-miss traffic of the 8-phase GEMM per tile raster (group_m), one shape at a time.

  rocprofv3 --pmc FETCH_SIZE -d OUT -o run --output-format csv -- python tools/raster_traffic.py run
  python tools/raster_traffic.py summarize OUT/run_counter_collection.csv

`run` launches REPS dispatches per (shape, group_m) in a fixed order; `summarize` maps the
dispatches back by order and prints FETCH_SIZE x 2 (the gfx950 correction of the MI355X guide)
per launch against the algorithmic bytes (X + W + Y [+ R]).
"""
import csv
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHAPES = {  # name: (M, N, K, resid)
    "mixer_cc": (50176, 768, 768, True),
    "mixer_up": (50176, 3072, 768, False),
    "mixer_down": (50176, 768, 3072, True),
    "enc_qkv": (51200, 2304, 768, False),
}
GROUPS = [1, 2, 4, 8, 16]
REPS = 3


def run():
    sys.path.insert(0, os.path.join(REPO, "sdp-net_amd"))
    import torch
    import sdpnet_hip as sp
    dev, bf = torch.device("cuda"), torch.bfloat16
    for name, (M, N, K, res) in SHAPES.items():
        x = torch.randn(M, K, device=dev).to(bf)
        w = (torch.randn(N, K, device=dev) * 0.05).to(bf)
        r = torch.randn(M, N, device=dev).to(bf) if res else None
        y = torch.empty(M, N, dtype=bf, device=dev)
        for gm in GROUPS:
            sp.lib().sdp_gemm_set_group_m(gm)
            for _ in range(REPS):
                sp.gemm(sp.dense(x), w, sp.dense(y), M, N, K, resid=None if r is None else sp.dense(r))
            torch.cuda.synchronize()
        del x, w, r, y
    sp.lib().sdp_gemm_set_group_m(-1)


def time_it():
    sys.path.insert(0, os.path.join(REPO, "sdp-net_amd"))
    import time
    import torch
    import sdpnet_hip as sp
    dev, bf = torch.device("cuda"), torch.bfloat16
    for name, (M, N, K, res) in SHAPES.items():
        x = torch.randn(M, K, device=dev).to(bf)
        w = (torch.randn(N, K, device=dev) * 0.05).to(bf)
        r = torch.randn(M, N, device=dev).to(bf) if res else None
        y = torch.empty(M, N, dtype=bf, device=dev)
        f = lambda: sp.gemm(sp.dense(x), w, sp.dense(y), M, N, K, resid=None if r is None else sp.dense(r))  # noqa: E731
        for gm in GROUPS + GROUPS:
            sp.lib().sdp_gemm_set_group_m(gm)
            t_end = time.time() + 0.3
            while time.time() < t_end:
                f()
                torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                f()
            e1.record()
            torch.cuda.synchronize()
            print(f"{name} group_m={gm}: {e0.elapsed_time(e1) * 50:.1f} us", flush=True)
    sp.lib().sdp_gemm_set_group_m(-1)


def summarize(path):
    rows = [r for r in csv.DictReader(open(path)) if "gemm_bf16_8ph" in r.get("Kernel_Name", "")]
    per = {}
    for r in rows:
        d = int(r["Dispatch_Id"])
        per[d] = per.get(d, 0.0) + float(r["Counter_Value"])
    disp = sorted(per)
    i = 0
    print("| shape | group_m | FETCH_SIZE x 2 per launch (MB) | algorithmic (MB) | ratio |")
    print("|---|---|---|---|---|")
    for name, (M, N, K, res) in SHAPES.items():
        alg = 2 * (M * K + N * K + M * N * (2 if res else 1)) / 1e6
        for gm in GROUPS:
            vals = [per[d] for d in disp[i:i + REPS]]
            i += REPS
            mb = 2 * 1024 * sum(vals) / len(vals) / 1e6
            print(f"| {name} | {gm} | {mb:.1f} | {alg:.1f} | {mb / alg:.2f} |")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    elif sys.argv[1] == "time":
        time_it()
    else:
        summarize(sys.argv[2])
