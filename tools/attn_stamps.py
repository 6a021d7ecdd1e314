"""Per-pair phase timeline of attn_fa4 / attn_fa5 / attn_fa6 (--shape xl) from the stamped diagnostic library.

  make -C sdp-net_amd/csrc stamps
  SDPNET_HIP_LIB=sdp-net_amd/lib_stamps/libsdpnet_hip.so python tools/attn_stamps.py [--shape m|xl]

Waves 0 and 3 of every workgroup record s_memtime (shader clock) at pair start, after the K/V
barrier, after the k-norm barrier and after each of the two query slots; printed as mean cycles
per phase, per pair index, plus the gap between a pair's end and the next pair's start.
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("SDPNET_HIP_LIB", os.path.join(REPO, "sdp-net_amd", "lib_stamps", "libsdpnet_hip.so"))
sys.path.insert(0, os.path.join(REPO, "sdp-net_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import sdpnet_hip as sp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="m", choices=["m", "xl"], help="m: bs 256, N 200; xl: bs 512, N 260")
    ap.add_argument("--kernel", type=int, default=4,
                    help="attention kernel tier (4: fa4, 6: fa5; 3 at --shape xl: fa6)")
    args = ap.parse_args()
    sp.lib().sdp_attention_set_kernel(args.kernel)
    B, N, H, hd = (256, 200, 8, 96) if args.shape == "m" else (512, 260, 8, 96)
    C = H * hd
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    qkv = torch.randn(B * N, 3 * C, generator=g).to(torch.bfloat16).to(dev)
    o = torch.empty(B * N, C, dtype=torch.bfloat16, device=dev)
    gq, bq, gk, bk = (torch.ones(hd, device=dev), torch.zeros(hd, device=dev), torch.ones(hd, device=dev),
                      torch.zeros(hd, device=dev))
    run = lambda: sp.attention(qkv, o, B, N, H, hd, qk_norm=(gq, bq, gk, bk), eps=1e-5)  # noqa: E731
    for _ in range(30):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        run()
    e1.record()
    torch.cuda.synchronize()
    print(f"attention {args.shape} shape: {1e3 * e0.elapsed_time(e1) / 20:.1f} us per launch (events), variant "
          f"{sp.attention_variant(torch.bfloat16, N, H, hd)}")
    L = sp.lib()
    buf = np.zeros(1024 * 2 * 8 * 5, dtype=np.uint64)
    L.sdp_attn_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    run()
    assert L.sdp_attn_stamps(buf.ctypes.data, buf.nbytes) == 0
    st = buf.reshape(1024, 2, 8, 5).astype(np.int64)
    if args.shape == "xl":  # attn_fa6: wave 0 / producer phases of one pair
        names = None
        waves = ["wave 0", "wave 11 (producer)"]
        wnames = [["k-norm", "barrier 2", "q + compute", "barrier 1"],
                  ["wait V", "barrier 2", "stage K+1", "barrier 1"]]
    elif args.kernel >= 6:  # attn_fa5: compute / produce, reach barrier 1, k-norm, barrier 2
        names, waves = ["work", "barrier 1", "k-norm", "barrier 2"], ["wave 0", "wave 7 (producer)"]
    else:
        names, waves = ["stage+wait", "k-norm", "slot 0", "slot 1"], ["wave 0", "wave 3"]
    for w, wn in enumerate(waves):
        if args.shape == "xl":
            names = wnames[w]
        print(f"  {wn}: mean cycles per phase by pair index (workgroups with that pair)")
        for j in range(8):
            ok = (st[:, w, j, :] != 0).all(axis=1)
            if not ok.any():
                continue
            d = np.diff(st[ok, w, j, :], axis=1)
            tot = st[ok, w, j, 4] - st[ok, w, j, 0]
            row = "  ".join(f"{n} {d[:, k].mean():7.0f}" for k, n in enumerate(names))
            gap = ""
            if j + 1 < 8:
                ok2 = ok & (st[:, w, j + 1, 0] != 0)
                if ok2.any():
                    gap = f"  -> next pair {np.mean(st[ok2, w, j + 1, 0] - st[ok2, w, j, 4]):6.0f}"
            print(f"    pair {j}: n={ok.sum():4d}  {row}  total {tot.mean():7.0f}{gap}")


if __name__ == "__main__":
    main()
