"""Solo timings of the training step's memory-bound kernels at SdP-Net-XL bs=120 shapes
(M = 120 x 256 image rows, C = 768, FFN 3072; fp32 residual stream, bf16 operands).

  python tools/train_kern_bench.py [--reps 50] [--only ln_bwd,act,rowscale,copy,add_ln]

Prints us per launch and the algorithmic bytes / time (GB/s) of each pass.
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
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--only", default="ln_bwd,act,rowscale,copy,add_ln")
    args = ap.parse_args()
    only = set(args.only.split(","))
    dev = torch.device("cuda")
    B, R, P, C = 120, 4, 256, 768
    N = R + P
    M = B * P
    f32, bf = torch.float32, torch.bfloat16
    Rows = sp.Rows

    def report(name, us, nbytes):
        print(f"{name:44s} {us:8.1f} us  {nbytes / 1e6:7.1f} MB  {nbytes / us / 1e6:6.2f} TB/s", flush=True)

    tok = torch.randn(B, N, C, device=dev)
    mid = torch.randn(B, N, C, device=dev)
    st = torch.stack([torch.randn(M, device=dev) * 0.1, torch.rand(M, device=dev) + 0.5], 1).contiguous()
    g = torch.randn(C, device=dev)
    bt = torch.randn(C, device=dev)
    da = torch.randn(M, C, device=dev).to(bf)
    img = lambda t: Rows(t, C, P, N, R)  # noqa: E731
    if "ln_bwd" in only:
        dmid = torch.empty_like(tok)
        z1 = torch.randn(M, C, device=dev).to(bf)
        dz1 = torch.empty(M, C, device=dev, dtype=bf)
        us = timeit(lambda: sp.ln_bwd(img(mid), st, g, sp.dense(da), img(dmid), M, C, add=img(tok)), args.reps)
        report("ln_bwd (fp32 x/add/dx, bf16 dy) + affine", us, M * C * 14)
        us = timeit(lambda: sp.ln_bwd(img(mid), st, g, sp.dense(da), img(dmid), M, C, add=img(tok), want_affine=False),
                    args.reps)
        report("ln_bwd, no affine partials", us, M * C * 14)
        us = timeit(lambda: sp.ln_bwd(img(mid), st, g, sp.dense(da), img(dmid), M, C, add=img(tok),
                                      emit=dict(out=dz1, z=z1, act=1)), args.reps)
        report("ln_bwd + affine + emit gelu' (mixer LN2)", us, M * C * 18)
    if "act" in only:
        z = torch.randn(M, 4 * C, device=dev).to(bf)
        h = torch.empty_like(z)
        dz = torch.empty_like(z)
        for p in (0.0, 0.2):
            us = timeit(lambda: sp.act_fwd(z, h, M, 4 * C, 1, p, 7), args.reps)
            report(f"act_fwd gelu p={p} [M, 4C]", us, M * 4 * C * 4)
            us = timeit(lambda: sp.act_bwd(z, h, dz, M, 4 * C, 1, p, 7), args.reps)
            report(f"act_bwd gelu p={p} [M, 4C]", us, M * 4 * C * 6)
    if "rowscale" in only:
        o = torch.empty(M, C, device=dev, dtype=bf)
        us = timeit(lambda: sp.rowscale_add(img(tok), sp.dense(o), M, C), args.reps)
        report("rowscale fp32 rows -> bf16 (dense copy)", us, M * C * 6)
        o32 = torch.empty_like(tok)
        z3 = torch.randn(M, C, device=dev).to(bf)
        us = timeit(lambda: sp.rowscale_add(sp.dense(z3), img(o32), M, C, resid=img(mid)), args.reps)
        report("rowscale bf16 + fp32 resid -> fp32", us, M * C * 10)
    if "copy" in only:
        dst = torch.empty_like(tok)
        us = timeit(lambda: sp.copy_rows(tok, C, N * C, dst, C, N * C, B, R, C), args.reps)
        report("copy register rows (fp32)", us, B * R * C * 8)
    if "add_ln" in only:
        z1 = torch.randn(M, C, device=dev).to(bf)
        a2 = torch.empty(M, C, device=dev, dtype=bf)
        s2 = torch.empty(M, 2, device=dev)
        us = timeit(lambda: sp.add_ln_fwd(sp.dense(z1), img(mid), sp.dense(a2), M, C, img(tok), 1e-6, g, bt, s2, act=1),
                    args.reps)
        report("add_ln_fwd gelu (bf16 z, fp32 resid/out, bf16 a)", us, M * C * 12)
        us = timeit(lambda: sp.ln_fwd(img(tok), 1e-6, g, bt, s2, sp.dense(a2), M, C), args.reps)
        report("ln_fwd fp32 -> bf16", us, M * C * 6)


if __name__ == "__main__":
    main()
