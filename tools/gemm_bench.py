"""Microbenchmark of sdp_gemm at the SdP-Net-M shapes (bs=256), random data.

  python tools/gemm_bench.py [--reps 20] [--streams 1,2]

Per shape: the production epilogue (bias / act / residual as the model uses it),
average µs per launch from HIP events, TFLOP/s.  With --streams 2 the same total
work is split into two half-M launches on two streams (tail filling).
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sdp-net_amd"))

import torch  # noqa: E402
import sdpnet_hip as sp  # noqa: E402

# name: (M, N, K, bias, act, resid, ln) -- the model's epilogues (sdp-net_amd/layers.py): a residual GEMM
# also writes the next LayerNorm's row partials; ln = LayerNorm folded in (row stats + weight column sums)
SHAPES = {
    "mixer_cc": (50176, 768, 768, True, 1, True, False),
    "mixer_up": (50176, 3072, 768, True, 1, False, True),
    "mixer_down": (50176, 768, 3072, True, 0, True, False),
    "enc_qkv": (51200, 2304, 768, True, 0, False, True),
    "enc_o": (51200, 768, 768, True, 0, True, False),
    "enc_ff1": (51200, 3072, 768, True, 1, False, True),
    "enc_ff2": (51200, 768, 3072, True, 0, True, False),
    "sq8192": (8192, 8192, 8192, False, 0, False, False),
    "mixer_up_noact": (50176, 3072, 768, True, 0, False, True),
    "mixer_cc_noact": (50176, 768, 768, True, 0, True, False),
    "mixer_cc_nores": (50176, 768, 768, True, 1, False, False),
}


def operands(name, g, dev):
    """Synthetic operands of one shape, the epilogue inputs the model passes (SHAPES)."""
    M, N, K, has_b, act, has_r, has_ln = SHAPES[name]
    bf = torch.bfloat16
    x = (torch.rand(M, K, generator=g) * 2 - 1).to(bf).to(dev)
    w = ((torch.rand(N, K, generator=g) * 2 - 1) * 0.05).to(bf).to(dev)
    b = torch.randn(N, generator=g).to(dev) if has_b else None
    r = torch.randn(M, N, generator=g).to(bf).to(dev) if has_r else None
    part = torch.empty(M, (N + 63) // 64, 2, device=dev) if has_r else None
    ln = None
    if has_ln:
        st = torch.stack([torch.randn(M, generator=g) * 0.1, torch.rand(M, generator=g) + 0.5], 1).to(dev)
        ln = (st.contiguous(), w.float().sum(1).contiguous())
    y = torch.empty(M, N, dtype=bf, device=dev)
    return M, N, K, act, x, w, b, r, part, ln, y


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--streams", default="1")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--kernels", default="14", help="bf16 fast kernel ids to A/B (9, 14)")
    ap.add_argument("--exact-gelu", default="0", help="GELU forms to A/B (0 tanh form, 1 exact erf)")
    ap.add_argument("--epi-spec", default="1", help="epilogue specialisation A/B (0 run-time flags, 1 compile-time)")
    ap.add_argument("--kloop", default="2", help="main-loop phases per K-tile A/B (4, 2)")
    ap.add_argument("--ct", default="0", help="cross-tile kernel settings to A/B: 'tiles[:re[:kmax]]' items, 0 = off")
    ap.add_argument("--warm-s", type=float, default=0.5, help="seconds of warm-up launches per variant")
    ap.add_argument("--torch", action="store_true", help="also time torch F.linear (hipBLASLt) as a yardstick")
    args = ap.parse_args()

    def combos():
        return [(kk, int(s_), int(d), c, int(e), int(kl)) for kk in args.kernels.split(",")
                for s_ in args.streams.split(",") for d in args.exact_gelu.split(",")
                for c in args.ct.split(",") for e in args.epi_spec.split(",") for kl in args.kloop.split(",")]
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    total_us = {}
    ref_out = {}
    for name in args.shapes.split(","):
        M, N, K, act, x, w, b, r, part, ln, y = operands(name, g, dev)
        for kern, ns, dsy, sch, spc, kl in combos():
            sp.lib().sdp_gemm_set_epi_spec(spc)
            sp.lib().sdp_gemm_set_kloop_phases(kl)
            sp.lib().sdp_gemm_set_fast_kernel(int(kern))
            sp.lib().sdp_gemm_set_exact_gelu(dsy)
            ct_t, ct_re, ct_k = (sch.split(":") + ["2", "1024"][len(sch.split(":")) - 1:])[:3]
            assert sp.lib().sdp_gemm_set_ct(int(ct_t), int(ct_re), int(ct_k), 1 << 30) >= -1
            streams = [torch.cuda.Stream() for _ in range(ns)]
            parts = []
            step = (M + ns - 1) // ns
            for i in range(ns):
                lo, hi = i * step, min(M, (i + 1) * step)
                parts.append((lo, hi))

            def run():
                cur = torch.cuda.current_stream()
                for s in streams:
                    s.wait_stream(cur)
                for s, (lo, hi) in zip(streams, parts):
                    with torch.cuda.stream(s):
                        sp.gemm(sp.dense(x[lo:hi]), w, sp.dense(y[lo:hi]), hi - lo, N, K, bias=b,
                                resid=None if r is None else sp.dense(r[lo:hi]), act=act,
                                ln=None if ln is None else (ln[0][lo:hi], ln[1]),
                                part=None if part is None else part[lo:hi])
                for s in streams:
                    cur.wait_stream(s)

            # warm up for ~0.5 s of GPU time so every variant is timed at the loaded clock
            # (the host-side tensor set-up leaves the GPU idle and down-clocked)
            import time
            t_end = time.time() + args.warm_s
            while time.time() < t_end:
                for _ in range(5):
                    run()
                torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = 1e3 * e0.elapsed_time(e1) / args.reps
            ref_y = ref_out.setdefault(name, y.clone())  # outputs must agree across kernels
            diff = float((y.float() - ref_y.float()).abs().max())
            tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
            total_us[(name, kern, ns, dsy, sch, spc, kl)] = us
            print(f"{name:11s} M={M:6d} N={N:5d} K={K:5d} kern={kern} ct={sch} streams={ns} exact_gelu={dsy} spec={spc} kloop={kl} "
                  f"{us:9.1f} us  {tf:7.1f} TF/s  ({100 * tf / 2516.6:4.1f}% of bf16 peak)  max|diff vs first| {diff:.3g}", flush=True)
        if args.torch:  # vendor-library yardstick (plain GEMM, no epilogue) -- not used by the product
            import torch.nn.functional as F
            f = lambda: F.linear(x, w)  # noqa: E731
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                f()
            e1.record()
            torch.cuda.synchronize()
            us = 1e3 * e0.elapsed_time(e1) / args.reps
            print(f"{name:11s} torch.F.linear (hipBLASLt, no epilogue) {us:9.1f} us  "
                  f"{2.0 * M * N * K / (us * 1e-6) / 1e12:7.1f} TF/s", flush=True)
    # per-forward estimate for M (launch counts per forward)
    counts = dict(mixer_cc=24, mixer_up=24, mixer_down=24, enc_qkv=13, enc_o=13, enc_ff1=13, enc_ff2=13)
    for key in combos():
        if all((n, *key) in total_us for n in counts):
            t = sum(total_us[(n, *key)] * c for n, c in counts.items())
            print(f"GEMM time per M forward (kernel, streams, exact_gelu, ct, spec, kloop = {key}): {t / 1e3:.2f} ms")


if __name__ == "__main__":
    main()
