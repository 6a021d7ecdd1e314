"""Training attention kernels at the SdP-Net-XL bs120 shape (B=120, N=260, H=8, hd=96).

  python tools/attn_train_bench.py [--p 0,0.2] [--reps 20]

Times the forward (attn_fwd_k) and the backward (attn_bwd_* kernels) with HIP events per call;
run it under `rocprofv3 --kernel-trace --stats` for the per-kernel split of the backward.
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
    ap.add_argument("--p", default="0,0.2")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--B", type=int, default=120)
    ap.add_argument("--N", type=int, default=260)
    args = ap.parse_args()
    B, N, H, hd = args.B, args.N, 8, 96
    C = H * hd
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    qkv = torch.randn(B * N, 3 * C, generator=g).to(torch.bfloat16).to(dev)
    do = torch.randn(B * N, C, generator=g).to(torch.bfloat16).to(dev)
    o = torch.empty(B * N, C, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * H * N, dtype=torch.float32, device=dev)
    delta = torch.empty(B * H * N, dtype=torch.float32, device=dev)
    dqkv = torch.empty(B * N, 3 * C, dtype=torch.bfloat16, device=dev)
    scale = hd ** -0.5
    # useful FLOPs per (b, h): forward S + PV, backward S, dP, dV, dK, dQ (no recompute counted twice)
    fl_fwd = 2 * 2 * N * N * hd * B * H
    fl_bwd = 5 * 2 * N * N * hd * B * H
    for p in [float(x) for x in args.p.split(",")]:
        fwd = lambda: sp.attn_train_fwd(qkv, o, lse, B, N, H, hd, scale, p, 1234)  # noqa: E731
        bwd = lambda: sp.attn_train_bwd(qkv, o, do, lse, delta, (dqkv, 0), (dqkv, C), (dqkv, 2 * C),  # noqa: E731
                                        B, N, H, hd, scale, p, 1234)
        fwd()
        tf = timeit(fwd, args.reps)
        tb = timeit(bwd, args.reps)
        print(f"p={p:.2f}  fwd {tf:8.1f} us ({fl_fwd / tf / 1e6:6.1f} TF/s)   bwd {tb:8.1f} us "
              f"({fl_bwd / tb / 1e6:6.1f} TF/s useful)   bwd/fwd {tb / tf:.2f}", flush=True)


if __name__ == "__main__":
    main()
