"""Solo timings of the training GEMM epilogues against GEMM + separate activation pass, at the
SdP-Net-XL bs120 FFN shapes (M = 30720 tokens, C = 768, hidden 3072), bf16.

  python tools/train_epi_bench.py [--reps 30]

mode 1 (forward):  z = x W^T + b, h = dropout(gelu(z))        vs  gemm + act_fwd
mode 2 (backward): dz = dropout(dy W) * gelu'(z)              vs  gemm (dh) + act_bwd
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sdp-net_amd"))
import torch  # noqa: E402
import sdpnet_hip as sp  # noqa: E402


def timeit(fn, reps):
    for _ in range(5):
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
    ap.add_argument("--reps", type=int, default=30)
    args = ap.parse_args()
    dev = torch.device("cuda")
    bf = torch.bfloat16
    M, C, H = 30720, 768, 3072
    g = torch.Generator(device="cpu").manual_seed(0)
    x = (torch.randn(M, C, generator=g) * 0.5).to(bf).to(dev)
    w1 = (torch.randn(H, C, generator=g) * 0.03).to(bf).to(dev)
    b1 = torch.randn(H, generator=g).to(dev) * 0.1
    z = torch.empty(M, H, device=dev, dtype=bf)
    h = torch.empty(M, H, device=dev, dtype=bf)
    dy = (torch.randn(M, C, generator=g) * 0.1).to(bf).to(dev)
    w2t = (torch.randn(H, C, generator=g) * 0.03).to(bf).to(dev)   # dX = dY W2: W2^T [H, C] as the GEMM's W
    dh = torch.empty(M, H, device=dev, dtype=bf)
    dz = torch.empty(M, H, device=dev, dtype=bf)
    flop = 2.0 * M * H * C
    for p in (0.0, 0.2):
        def sep1():
            sp.gemm(sp.dense(x), w1, sp.dense(z), M, H, C, bias=b1)
            sp.act_fwd(z, h, M, H, 1, p, 5)
        t_g = timeit(lambda: sp.gemm(sp.dense(x), w1, sp.dense(z), M, H, C, bias=b1), args.reps)
        t_s = timeit(sep1, args.reps)
        t_f = timeit(lambda: sp.gemm_train_epi(1, x, w1, z, M, H, C, bias=b1, y2=h, act=1, p=p, seed=5), args.reps)
        print(f"mode 1 p={p}: gemm {t_g:7.1f} us ({flop / t_g / 1e6:6.1f} TF/s)  gemm+act_fwd {t_s:7.1f} us  "
              f"fused {t_f:7.1f} us", flush=True)

        def sep2():
            sp.gemm(sp.dense(dy), w2t, sp.dense(dh), M, H, C)
            sp.act_bwd(z, dh, dz, M, H, 1, p, 5)
        t_g = timeit(lambda: sp.gemm(sp.dense(dy), w2t, sp.dense(dh), M, H, C), args.reps)
        t_s = timeit(sep2, args.reps)
        t_f = timeit(lambda: sp.gemm_train_epi(2, dy, w2t, dz, M, H, C, z=z, act=1, p=p, seed=5), args.reps)
        print(f"mode 2 p={p}: gemm {t_g:7.1f} us ({flop / t_g / 1e6:6.1f} TF/s)  gemm+act_bwd {t_s:7.1f} us  "
              f"fused {t_f:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
