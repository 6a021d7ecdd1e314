"""Throughput of the evaluation ends of the path.

  python tools/eval_bench.py [--batch 256] [--reps 20] [--hw 375,500]

* sdp_val_preprocess on a device-resident batch of decoded uint8 images (ImageNet-like
  375 x 500 by default) -> [B, 3, 224, 224] fp32: images/s and GB/s against the HBM
  roofline, algorithmic bytes = input pixels read once + output written once.
* sdp_logits_metrics on [B, 1000] logits.
* CPU baseline: the reference's per-image transform chain (Pillow resize + crop, then
  /255 and Normalize in numpy) on one host core, a bounded sample.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sdp-net_amd"))

import torch  # noqa: E402

import sdpnet_hip as sp  # noqa: E402
import preprocess  # noqa: E402

HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--hw", default="375,500")
    ap.add_argument("--cpu-images", type=int, default=64)
    args = ap.parse_args()
    H, W = (int(v) for v in args.hw.split(","))
    B = args.batch
    rng = np.random.default_rng(0)
    imgs = [rng.integers(0, 256, (H, W, 3), dtype=np.uint8) for _ in range(B)]
    t = preprocess.val_transforms()
    dev = torch.device("cuda")
    # device-resident packed batch (the timed region excludes the host packing / H2D copy)
    pix = torch.from_numpy(np.concatenate([a.reshape(-1) for a in imgs])).to(dev)
    offs = torch.arange(B, dtype=torch.int64, device=dev) * (H * W * 3)
    hw = torch.tensor([[H, W]] * B, dtype=torch.int32, device=dev)
    kmax = max(preprocess._taps(W, 320), preprocess._taps(H, 320))

    def run():
        return sp.val_preprocess(pix, offs, hw, (320, 320), (224, 224), t.top, t.left, kmax, t.mean, t.std,
                                 H * 224 * 4, torch.float32, max_w=W)[0]

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = 1e3 * e0.elapsed_time(e1) / args.reps
    algo = B * (H * W * 3 + 3 * 224 * 224 * 4)
    gbs = algo / (us * 1e-6) / 1e9
    pre = {"op": "sdp_val_preprocess", "batch": B, "image_hw": [H, W], "us_per_batch": round(us, 2),
           "images_per_s": round(B / (us * 1e-6), 1), "algorithmic_bytes_per_batch": algo,
           "achieved_GBs": round(gbs, 1), "hbm_peak_GBs": HBM_PEAK_GBS, "frac": round(gbs / HBM_PEAK_GBS, 4)}
    # end-to-end from host images (packing + pinned H2D copy + kernels), for reference
    t0 = time.perf_counter()
    n_e2e = 3
    for _ in range(n_e2e):
        t(imgs)
    torch.cuda.synchronize()
    pre["host_to_device_images_per_s"] = round(n_e2e * B / (time.perf_counter() - t0), 1)

    logits = torch.randn(B, 1000, device=dev)
    labels = torch.randint(0, 1000, (B,), device=dev)
    for _ in range(3):
        sp.logits_metrics(logits, labels)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(args.reps):
        sp.logits_metrics(logits, labels)
    e1.record()
    torch.cuda.synchronize()
    mus = 1e3 * e0.elapsed_time(e1) / args.reps
    met = {"op": "sdp_logits_metrics", "batch": B, "classes": 1000, "us_per_batch": round(mus, 2),
           "achieved_GBs": round(B * 1000 * 4 / (mus * 1e-6) / 1e9, 1)}

    # CPU baseline: Pillow resize + crop + normalize per image, one core
    from PIL import Image
    mean = np.array(preprocess.IMAGENET_MEAN, np.float32)[:, None, None]
    std = np.array(preprocess.IMAGENET_STD, np.float32)[:, None, None]
    n = min(args.cpu_images, B)
    t0 = time.perf_counter()
    for a in imgs[:n]:
        r = np.asarray(Image.fromarray(a).resize((320, 320), Image.BICUBIC))[48:272, 48:272]
        x = r.transpose(2, 0, 1).astype(np.float32) / 255.0
        _ = (x - mean) / std
    cpu = n / (time.perf_counter() - t0)
    pre["cpu_baseline"] = {"value": round(cpu, 1), "unit": "images/s", "cores": 1, "kind": "port",
                           "sample": f"{n} images {H}x{W}, Pillow resize + numpy normalize"}
    print(json.dumps(pre))
    print(json.dumps(met))


if __name__ == "__main__":
    main()
