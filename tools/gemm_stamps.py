"""Per-workgroup timeline of the 8-phase GEMM from the stamped diagnostic library.

  make -C sdp-net_amd/csrc stamps
  python tools/gemm_stamps.py [--shapes mixer_cc,mixer_up] [--schedules 0,1]

Loads sdp-net_amd/lib_stamps/libsdpnet_hip.so (built with -DSDP_GEMM_STAMPS: every
workgroup records s_memrealtime at its start, each segment start, after the prologue
wait, after the k-loop, after the epilogue / partial store, and around a stream-K wait)
and prints, per shape and schedule, the mean time of each part per segment and how many
workgroups are in their epilogue at once (the store bursts).
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
from gemm_bench import SHAPES  # noqa: E402

TICK_US = 0.01  # s_memrealtime runs at 100 MHz


def read_stamps(nwg):
    buf = np.zeros(8192 * 64, dtype=np.uint64)
    L = sp.lib()
    fn = L.sdp_gemm_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]
    fn.restype = ctypes.c_int
    assert fn(buf.ctypes.data, buf.nbytes, 1) == 0
    return buf.reshape(8192, 64)[:nwg]


def analyse(st, label):
    codes = (st >> np.uint64(56)).astype(np.int64)
    t = (st & np.uint64((1 << 56) - 1)).astype(np.int64)
    valid = st != 0
    t0 = t[valid].min()
    tend = t[valid].max()
    parts = {"prologue": [], "kloop": [], "epilogue": [], "head_store": [], "tail_wait": []}
    epi_iv = []
    nseg = []
    for w in range(st.shape[0]):
        ev = [(int(c), int(x) - t0) for c, x, v in zip(codes[w], t[w], valid[w]) if v]
        if not ev:
            continue
        nseg.append(sum(1 for c, _ in ev if c >= 0x10))
        mode, last = None, {}
        for c, x in ev:
            if c >= 0x10:
                mode = c - 0x10
                last = {"seg": x}
            elif c == 2:
                last["p0"] = x
            elif c == 3:
                parts["tail_wait"].append(x - last["p0"])
            elif c == 4:
                parts["prologue"].append(x - last["seg"])
                last["k"] = x
            elif c == 5:
                parts["kloop"].append(x - last["k"])
                last["e"] = x
            elif c == 6:
                (parts["head_store"] if mode == 1 else parts["epilogue"]).append(x - last["e"])
                if mode != 1:
                    epi_iv.append((last["e"], x))
    span = (tend - t0) * TICK_US
    print(f"  {label}: span {span:.1f} us over {st.shape[0]} workgroups, segments/wg {np.mean(nseg):.2f}")
    for k, v in parts.items():
        if v:
            a = np.array(v) * TICK_US
            print(f"    {k:11s} n={len(a):5d} mean {a.mean():7.2f} us  p10 {np.percentile(a, 10):7.2f}  "
                  f"p90 {np.percentile(a, 90):7.2f}  max {a.max():7.2f}")
    if epi_iv:  # workgroups inside an epilogue, sampled every 1 us
        nb = int(span) + 1
        occ = np.zeros(nb)
        for a, b in epi_iv:
            occ[int(a * TICK_US):int(b * TICK_US) + 1] += 1
        print("    in-epilogue count per us:", " ".join(str(int(o)) for o in occ))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="mixer_cc,mixer_up,mixer_down,enc_qkv")
    ap.add_argument("--schedules", default="0")
    ap.add_argument("--dephase", default="0", help="first-round start offsets per group of 8 workgroups per XCD, "
                    "in 10-ns ticks (experiment: group g = (b >> 3) & 3 waits g * value)")
    args = ap.parse_args()
    L = sp.lib()
    L.sdp_gemm_set_dephase.argtypes = [ctypes.c_int]
    dev = torch.device("cuda")
    bf = torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(0)
    for name in args.shapes.split(","):
        M, N, K, has_b, act, has_r = SHAPES[name]
        x = (torch.rand(M, K, generator=g) * 2 - 1).to(bf).to(dev)
        w = ((torch.rand(N, K, generator=g) * 2 - 1) * 0.05).to(bf).to(dev)
        b = torch.randn(N, generator=g).to(dev) if has_b else None
        r = torch.randn(M, N, generator=g).to(bf).to(dev) if has_r else None
        y = torch.empty(M, N, dtype=bf, device=dev)
        print(f"{name} M={M} N={N} K={K}")
        for sch, dph in [(int(c), int(d)) for c in args.schedules.split(",") for d in args.dephase.split(",")]:
            assert L.sdp_gemm_set_dephase(dph) == 0
            run = lambda: sp.gemm(sp.dense(x), w, sp.dense(y), M, N, K, bias=b,  # noqa: E731
                                  resid=None if r is None else sp.dense(r), act=act)
            for _ in range(30):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                run()
            e1.record()
            torch.cuda.synchronize()
            print(f"  dephase {dph} ticks: {1e3 * e0.elapsed_time(e1) / 20:.1f} us per launch (events)")
            read_stamps(1)
            run()
            sk = 0
            nwg = 256 if sk else ((M + 255) // 256) * ((N + 255) // 256)
            analyse(read_stamps(nwg), f"schedule {sch} ({'stream-K' if sk else 'data-parallel'})")


if __name__ == "__main__":
    main()
