"""Microbenchmark of the non-GEMM kernels at SdP-Net-M (bs=256) or -XL (bs=512) shapes, bf16.

  python tools/kern_bench.py [--reps 20] [--only dw,attn,ln,stats] [--shape m|xl] [--attn-kerns 2,3,4,5]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sdp-net_amd"))
import torch  # noqa: E402
import sdpnet_hip as sp  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return 1e3 * e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="dw,attn,ln,stats")
    ap.add_argument("--attn-kerns", default="3,4,5")
    ap.add_argument("--shape", default="m", choices=["m", "xl"], help="M: bs 256, 14x14 patches; XL: bs 512, 16x16")
    args = ap.parse_args()
    dev, bf = "cuda", torch.bfloat16
    B, R, H, W, C, heads = (256, 4, 14, 14, 768, 8) if args.shape == "m" else (512, 4, 16, 16, 768, 8)
    P, N = H * W, R + H * W
    only = args.only.split(",")
    tok = torch.randn(B * N, C, device=dev).to(bf)
    img = sp.Rows(tok, C, P, N, R)
    if "stats" in only or "dw" in only:
        stats = torch.empty(B * P, 2, device=dev)
        us = timeit(lambda: sp.rowstats(img, 1e-6, stats, B * P, C), args.reps)
        print(f"rowstats   {us:8.1f} us  {B * P * C * 2 / us / 1e3:7.1f} GB/s (read)")
    if "dw" in only:
        w = torch.randn(C, 49, device=dev) * 0.1
        g, be = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        y = torch.empty(B * P, C, device=dev, dtype=bf)
        for kern in (1, 2, 3):
            old = sp.lib().sdp_dwconv_set_kernel(kern)
            us = timeit(lambda: sp.dwconv(img, w, None, sp.dense(y), B, H, W, C, 7, stats=stats, ln_gamma=g,
                                          ln_beta=be), args.reps)
            sp.lib().sdp_dwconv_set_kernel(old)
            print(f"dwconv_ln k{kern} {us:8.1f} us  {2 * B * P * C * 2 / us / 1e3:7.1f} GB/s (read+write)")
    if "ln" in only:
        g, be = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        y = torch.empty(B * N, C, device=dev, dtype=bf)
        us = timeit(lambda: sp.layernorm(sp.dense(tok), g, be, 1e-5, sp.dense(y), B * N, C), args.reps)
        print(f"layernorm  {us:8.1f} us  {2 * B * N * C * 2 / us / 1e3:7.1f} GB/s (read+write)")
    if "attn" in only:
        hd = C // heads
        qkv = torch.randn(B * N, 3 * C, device=dev).to(bf)
        o = torch.empty(B * N, C, device=dev, dtype=bf)
        g = torch.ones(hd, device=dev)
        z = torch.zeros(hd, device=dev)
        for kern in [int(k) for k in args.attn_kerns.split(",")]:
            old = sp.lib().sdp_attention_set_kernel(kern)
            us = timeit(lambda: sp.attention(qkv, o, B, N, heads, hd, qk_norm=(g, z, g, z)), args.reps)
            sp.lib().sdp_attention_set_kernel(old)
            fl = 4.0 * B * heads * N * N * hd
            by = B * N * 4 * C * 2
            print(f"attention k{kern} {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s  {by / us / 1e3:7.1f} GB/s")


if __name__ == "__main__":
    main()
