"""Phase timeline of the 8-phase GEMM main loop (diagnostic library only).

  make -C sdp-net_amd/csrc stamps
  python tools/gemm_phases.py [--shapes mixer_down,enc_qkv]

Workgroup 0's waves 0 (group 0) and 4 (group 1) stamp s_memtime (shader clock) and s_memrealtime
(100 MHz) at every MFMA
section's start (after its barrier and lgkmcnt wait) and after its last MFMA issue, for the first
8 K-tiles (stamps build, sdp-net_amd/lib_stamps; never loaded by the product).  Prints per phase
of each K-tile: the MFMA section length of each group (16 MFMAs = 256 cycles of issue at one
MFMA / 16 cycles) and the gap from one group's section end to the other group's next start.
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("SDPNET_HIP_LIB", os.path.join(REPO, "sdp-net_amd", "lib_stamps", "libsdpnet_hip.so"))
sys.path.insert(0, os.path.join(REPO, "sdp-net_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import sdpnet_hip as sp  # noqa: E402
from gemm_bench import operands  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="mixer_down,enc_qkv,mixer_cc")
    args = ap.parse_args()
    L = sp.lib()
    L.sdp_gemm_phase_stamps.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    for name in args.shapes.split(","):
        M, N, K, act, x, w, b, r, part, ln, y = operands(name, g, dev)
        run = lambda: sp.gemm(sp.dense(x), w, sp.dense(y), M, N, K, bias=b,  # noqa: E731
                              resid=None if r is None else sp.dense(r), act=act, ln=ln, part=part)
        for _ in range(30):
            run()
        torch.cuda.synchronize()
        run()
        buf = np.zeros(256, dtype=np.uint64)
        assert L.sdp_gemm_phase_stamps(buf.ctypes.data) == 0
        st = buf[:128].reshape(2, 64).astype(np.int64)
        rt = buf[128:].reshape(2, 64).astype(np.int64)
        nph = L.sdp_gemm_set_kloop_phases(0)  # MFMA sections per K-tile (0: query only)
        t0 = min(st[0, 0], st[1, 0])
        st = st - t0
        print(f"{name} M={M} N={N} K={K}  (cycles from group 0's first MFMA section)")
        print("  kt ph | g0 start  len | g1 start  len | g0end->g1start  g1end->g0next")
        for i in range(8 * nph):
            kt, ph = divmod(i, nph)
            a0, e0 = st[0, 2 * i], st[0, 2 * i + 1]
            a1, e1 = st[1, 2 * i], st[1, 2 * i + 1]
            nx = st[0, 2 * i + 2] if i < 8 * nph - 1 else e1
            print(f"  {kt:2d} {ph:2d} | {a0:8d} {e0 - a0:4d} | {a1:8d} {e1 - a1:4d} | {a1 - e0:8d} {nx - e1:12d}")
        per = (st[0, 2 * 7 * nph] - st[0, 2 * nph]) / 6
        print(f"  mean cycles per K-tile (both groups' sections) over K-tiles 1..6: {per:.0f} (MFMA floor 2048)")
        last = 31  # the second s_memrealtime stamp
        ghz = (st[0, last] - st[0, 0]) / max(1, rt[0, last] - rt[0, 0]) * 0.1  # s_memrealtime: 100 MHz
        print(f"  shader clock over the 8 K-tiles (s_memtime / s_memrealtime): {ghz:.2f} GHz")


if __name__ == "__main__":
    main()
