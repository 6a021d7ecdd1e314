"""Step-time bound of the non-GEMM kernels (timing experiment; results are WRONG while skipping).

  python tools/skip_bench.py [--masks 0,1,2,4,7] [--reps 30]

For each sdp_debug_skip mask (bit 0 depthwise conv, bit 1 attention, bit 2 LN statistics) the
SdP-Net-M bs-256 bf16 forward (bench.py's model, 2 sub-batch streams) is captured into a HIP graph
and replayed; the drop in ms per step bounds what a faster kernel of that kind could give.  Masks are
interleaved twice.
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sdp-net_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--masks", default="0,1,2,4,7")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--config", default="m")
    args = ap.parse_args()
    import bench
    import model as sdp
    import sdpnet_hip as sp
    C = bench.CONFIGS[args.config]
    dev = torch.device("cuda")
    torch.manual_seed(231424314)
    m = sdp.MainModel.from_dict(**C["cfg"]).eval().to(dev)
    x = torch.randn(C["batch"], 3, 224, 224, generator=torch.Generator().manual_seed(1000)).to(dev).to(torch.bfloat16)
    res = {}
    for rnd in range(2):
        for mask in [int(v) for v in args.masks.split(",")]:
            sp.lib().sdp_debug_skip(mask)
            for _ in range(3):
                m(x)
            torch.cuda.synchronize()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                m(x)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                m(x)
            for _ in range(5):
                g.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                g.replay()
            torch.cuda.synchronize()
            ms = 1e3 * (time.perf_counter() - t0) / args.reps
            res.setdefault(mask, []).append(ms)
            print(f"round {rnd} skip mask {mask}: {ms:.3f} ms per step", flush=True)
            del g
    sp.lib().sdp_debug_skip(0)
    base = min(res[0])
    for mask, v in res.items():
        print(f"mask {mask} (dwconv={mask & 1}, attention={(mask >> 1) & 1}, ln_stats={(mask >> 2) & 1}): "
              f"best {min(v):.3f} ms, saves {base - min(v):.3f} ms of {base:.3f}")


if __name__ == "__main__":
    main()
