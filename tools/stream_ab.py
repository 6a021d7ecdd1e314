"""A/B of sub-batch stream schedules for the SdP-Net-M bf16 forward (bs 256, one GPU).

  python tools/stream_ab.py [--rounds 4] [--reps 30] [--configs default,contig,inter,off10]

Each config is captured as its own HIP graph of one forward; the graphs are replayed in
interleaved rounds (one process, same weights / inputs) and the median img/s per config is
printed.  Configs: default (2 plain streams), contig / inter (2 streams restricted to disjoint
CU halves, sdp_stream_create_cu_mask), offN (stream 1 starts N us after stream 0), and
combinations such as contig+off10 or s3 (3 streams).
"""
import argparse
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sdp-net_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--configs", default="default,contig,inter,off10,off25,contig+off10")
    args = ap.parse_args()
    import model as sdp
    dev = torch.device("cuda")
    sys.path.insert(0, REPO)
    from bench import M_CFG as cfg  # the headline workload (BASELINE.json configs[1])
    torch.manual_seed(231424314)
    m = sdp.MainModel.from_dict(**cfg).eval().to(dev)
    g = torch.Generator(device="cpu").manual_seed(1000)
    x = torch.randn(args.batch, 3, 224, 224, generator=g).to(dev).to(torch.bfloat16)
    graphs, outs = {}, {}
    for name in args.configs.split(","):
        parts = name.split("+")
        m.cu_split = next((p for p in parts if p in ("contig", "inter")), None)
        m.stream_offset_us = next((float(p[3:]) for p in parts if p.startswith("off")), 0.0)
        m.num_streams = next((int(p[1:]) for p in parts if p.startswith("s") and p[1:].isdigit()), 2)
        for _ in range(3):
            m(x)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            outs[name] = m(x)
        gr.replay()
        torch.cuda.synchronize()
        graphs[name] = gr
    ref = next(iter(outs.values())).float()
    for name, o in outs.items():
        print(f"{name}: max|logits - first| {(o.float() - ref).abs().max().item():.3e}", flush=True)
    res = {n: [] for n in graphs}
    for r in range(args.rounds):
        for name, gr in graphs.items():
            for _ in range(3):
                gr.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                gr.replay()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.reps
            res[name].append(args.batch / dt)
        print(f"round {r}: " + "  ".join(f"{n} {v[-1]:.0f}" for n, v in res.items()), flush=True)
    for name, v in res.items():
        print(f"{name:16s} median {statistics.median(v):8.1f} img/s  min {min(v):8.1f}  max {max(v):8.1f}")


if __name__ == "__main__":
    main()
