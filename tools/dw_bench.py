"""Microbenchmark of the training weight gradient dW = dY^T X (sdpnet_train._wgrad: gemm_flex
split-K into fp32 slabs + seg_colsum) at the SdP-Net-XL bs120 shapes, random bf16 data.

  python tools/dw_bench.py [--reps 20] [--impl flex,w8]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sdp-net_amd"))

import torch  # noqa: E402

# name: (tokens M, N_out, K_in)
SHAPES = {
    "cc": (30720, 768, 768),
    "up": (30720, 3072, 768),
    "down": (30720, 768, 3072),
    "qkv": (31200, 2304, 768),
    "o": (31200, 768, 768),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--impl", default="flex,8ph")
    args = ap.parse_args()
    import sdpnet_train as st
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    for name in args.shapes.split(","):
        M, N, K = SHAPES[name]
        dy = (torch.randn(M, N, generator=g) * 0.1).to(torch.bfloat16).to(dev)
        x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(dev)
        ref = None
        for impl in args.impl.split(","):
            st._WGRAD_8PH = impl != "flex"
            fn = st._wgrad
            for _ in range(5):
                out = fn(dy, x)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                out = fn(dy, x)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.reps
            tf = 2.0 * M * N * K / us * 1e-6
            if ref is None:
                ref = (dy.float().t() @ x.float())
            err = (out - ref).abs().max().item() / max(1e-6, ref.abs().max().item())
            print(f"{name:5s} M={M} N={N} K={K} {impl:5s} {us:8.1f} us {tf:7.1f} TF/s  rel err {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
