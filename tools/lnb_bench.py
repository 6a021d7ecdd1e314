"""Microbenchmark of the training LayerNorm backward at the SdP-Net-XL bs120 shape (fp32 stream x and
addend, bf16 dy, C = 768): python tools/lnb_bench.py [--reps 50]  (SDPNET_HIP_LIB selects a library)."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sdp-net_amd"))
import torch  # noqa: E402
import sdpnet_hip as sp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda")
    M, C = 31200, 768
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(M, C, generator=g).to(dev)
    dy = torch.randn(M, C, generator=g).to(torch.bfloat16).to(dev)
    add = torch.randn(M, C, generator=g).to(dev)
    st = torch.stack([x.mean(1), (x.var(1, unbiased=False) + 1e-5).rsqrt()], 1).contiguous()
    gam = torch.rand(C, generator=g).to(dev) + 0.5
    dx = torch.empty(M, C, device=dev)
    for rep in range(3):
        for _ in range(5):
            sp.ln_bwd(sp.dense(x), st, gam, sp.dense(dy), sp.dense(dx), M, C, add=sp.dense(add))
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            sp.ln_bwd(sp.dense(x), st, gam, sp.dense(dy), sp.dense(dx), M, C, add=sp.dense(add))
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.reps
        nb = M * C * (4 + 2 + 4 + 4)
        print(f"ln_bwd fp32 stream M={M} C={C}: {us:7.1f} us  {nb / us / 1e3:7.1f} GB/s  "
              f"dx checksum {float(dx.double().sum()):.6e}", flush=True)


if __name__ == "__main__":
    main()
