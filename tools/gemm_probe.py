"""Probe: is the bf16 GEMM main loop bound by operand fetch or by its own schedule?
Times the no-store kernel (id 10) on the M shapes with X dense (streams 77-308 MB
from HBM/MALL) vs X aliased to 256 rows (RowMap grp=256, gstride=0: one tile's rows,
L2-resident), same grid and instruction stream."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sdp-net_amd"))
import torch  # noqa: E402
import sdpnet_hip as sp  # noqa: E402

SH = [(50176, 768, 768), (50176, 3072, 768), (50176, 768, 3072), (8192, 8192, 8192)]
bf = torch.bfloat16
DIST = {"normal": lambda *s: torch.randn(*s, device="cuda"),
        "uniform": lambda *s: torch.rand(*s, device="cuda") * 2 - 1,
        "zeros": lambda *s: torch.zeros(*s, device="cuda")}
for kern, dist in [(int(k), d) for k in os.environ.get("PROBE_KERNELS", "10,12").split(",")
                   for d in os.environ.get("PROBE_DIST", "normal").split(",")]:
    sp.lib().sdp_gemm_set_fast_kernel(kern)
    for M, N, K in SH:
        x = DIST[dist](M, K).to(bf)
        w = (DIST[dist](N, K) * 0.05).to(bf)
        y = torch.empty(M, N, device="cuda", dtype=bf)
        res = {}
        for name, xr in (("dense", sp.Rows(x, K)), ("hotX", sp.Rows(x, K, 256, 0, 0))):
            f = lambda: sp.gemm(xr, w, sp.dense(y), M, N, K)  # noqa: E731
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                f()
            e1.record()
            torch.cuda.synchronize()
            res[name] = 1e3 * e0.elapsed_time(e1) / 20
        if os.environ.get("PROBE_TORCH"):  # vendor yardstick: torch F.linear (hipBLASLt), same timing loop
            f = lambda: torch.nn.functional.linear(x, w)  # noqa: E731
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            e0.record()
            for _ in range(20):
                f()
            e1.record()
            torch.cuda.synchronize()
            res["hipBLASLt"] = 1e3 * e0.elapsed_time(e1) / 20
        tf = {k: 2.0 * M * N * K / (v * 1e-6) / 1e12 for k, v in res.items()}
        print(f"kern={kern} {dist:7s} {M}x{N}x{K}: dense {res['dense']:.1f} us ({tf['dense']:.0f} TF/s)  "
              f"hotX {res['hotX']:.1f} us ({tf['hotX']:.0f} TF/s)"
              + (f"  hipBLASLt {res['hipBLASLt']:.1f} us ({tf['hipBLASLt']:.0f} TF/s)" if "hipBLASLt" in res else ""),
              flush=True)
