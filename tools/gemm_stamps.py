"""Per-workgroup timeline of the 8-phase GEMM from the stamped diagnostic library.

  make -C sdp-net_amd/csrc stamps
  python tools/gemm_stamps.py [--shapes mixer_cc,mixer_up] [--epi-wait 0,1]

Loads sdp-net_amd/lib_stamps/libsdpnet_hip.so (built with -DSDP_GEMM_STAMPS: every
workgroup records s_memrealtime at its start, each segment start, after the prologue
wait, after the k-loop, after the epilogue; wave 0 also stamps the epilogue's parts)
and prints, per shape, the mean time of each part per segment and how many
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
from gemm_bench import operands  # noqa: E402

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
        ev = [(int(c), int(x) - t0) for c, x, v in zip(codes[w][:40], t[w][:40], valid[w][:40]) if v]
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
    # epilogue sub-phases (fast epilogue only): slots 40.. hold codes 0x20 + k
    es = st[:, 40:45]
    if (es != 0).all(axis=1).any():
        ok = (es != 0).all(axis=1)
        et = (es[ok] & np.uint64((1 << 56) - 1)).astype(np.int64)
        names = ["resid loads", "stage", "LDS read-back", "drain + stores"]
        print("    epilogue parts (wave 0): " + ", ".join(
            f"{n} {np.mean(et[:, k + 1] - et[:, k]) * TICK_US:.2f}" for k, n in enumerate(names)) + " us")
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
    ap.add_argument("--epi-wait", default="0", help="1: drain memory counters before each epilogue stamp")
    ap.add_argument("--dephase", default="0", help="first-round start offsets per group of 8 workgroups per XCD, "
                    "in 10-ns ticks (experiment: group g = (b >> 3) & 3 waits g * value)")
    args = ap.parse_args()
    L = sp.lib()
    L.sdp_gemm_set_dephase.argtypes = [ctypes.c_int]
    L.sdp_gemm_set_epi_wait.argtypes = [ctypes.c_int]
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    for name in args.shapes.split(","):
        M, N, K, act, x, w, b, r, part, ln, y = operands(name, g, dev)
        print(f"{name} M={M} N={N} K={K}")
        for ew, dph in [(int(c), int(d)) for c in args.epi_wait.split(",") for d in args.dephase.split(",")]:
            assert L.sdp_gemm_set_dephase(dph) == 0
            assert L.sdp_gemm_set_epi_wait(ew) == 0
            run = lambda: sp.gemm(sp.dense(x), w, sp.dense(y), M, N, K, bias=b,  # noqa: E731
                                  resid=None if r is None else sp.dense(r), act=act, ln=ln, part=part)
            for _ in range(30):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                run()
            e1.record()
            torch.cuda.synchronize()
            print(f"  epi_wait {ew} dephase {dph} ticks: {1e3 * e0.elapsed_time(e1) / 20:.1f} us per launch (events)")
            read_stamps(1)
            run()
            nwg = ((M + 255) // 256) * ((N + 255) // 256)
            analyse(read_stamps(nwg), f"epi_wait {ew}")


if __name__ == "__main__":
    main()
