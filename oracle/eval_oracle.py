"""CPU oracle for the evaluation ends of the path — TEST INFRASTRUCTURE ONLY.

Restates, in numpy / stock torch CPU ops:

* the reference's validation transform ``val_transforms`` (hf_dataset_generator.py:27-41,
  used by model_test.py:50-52): RGB -> Resize((320, 320), BICUBIC) -> CenterCrop(224)
  -> ToDtype(float32, scale=True) -> Normalize(ImageNet mean / std).  For PIL images
  torchvision hands the resize to Pillow (a third-party dependency absent from
  /root/reference; the container pins Pillow 12.2.0).  ``pil_resize_u8`` restates Pillow's
  published 8-bit resampler (libImaging/Resample.c: precompute_coeffs, bicubic_filter
  with a = -0.5, normalize_coeffs_8bpc, ImagingResampleHorizontal/Vertical_8bpc,
  ImagingResampleInner's pass skipping).  It is pinned bit for bit against Pillow itself
  in tests/test_eval_oracle.py; CenterCrop's origin is torchvision's
  ``int(round((size - crop) / 2.0))`` (torchvision is not installed here: that formula
  and ToDtype/Normalize's x / 255, (x - mean) / std are restated from its published code,
  parity unpinned at the last fp32 ulp).
* ``run_test``'s metrics (model_test.py:69-85): nn.CrossEntropyLoss, the
  BCEWithLogitsLoss closure of training_utilities.py:95-107 and top-1 accuracy.

Who may use it: ``tests/`` only, as the checker.  The product path never imports it.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

PRECISION_BITS = 32 - 8 - 2  # Resample.c
IMAGENET_MEAN = (0.485, 0.456, 0.406)  # hf_dataset_generator.py:30-31
IMAGENET_STD = (0.229, 0.224, 0.225)


def _bicubic(x: float) -> float:
    """Resample.c bicubic_filter, a = -0.5."""
    a = -0.5
    if x < 0.0:
        x = -x
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def _c_int(v: float) -> int:
    """C (int) conversion of a double: truncation toward zero."""
    return int(math.trunc(v))


def precompute_coeffs(in_size: int, out_size: int):
    """Resample.c precompute_coeffs(inSize, 0, inSize, outSize, bicubic) followed by
    normalize_coeffs_8bpc: dense int64 matrix [out_size, in_size] of 22-bit taps."""
    scale = filterscale = in_size / out_size
    if filterscale < 1.0:
        filterscale = 1.0
    support = 2.0 * filterscale
    ss = 1.0 / filterscale
    K = np.zeros((out_size, in_size), dtype=np.int64)
    for xx in range(out_size):
        center = 0.0 + (xx + 0.5) * scale
        xmin = _c_int(center - support + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = _c_int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        ws = [_bicubic((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = 0.0
        for w in ws:
            ww += w
        for x, w in enumerate(ws):
            if ww != 0.0:
                w = w / ww
            K[xx, xmin + x] = _c_int(-0.5 + w * (1 << PRECISION_BITS)) if w < 0 else _c_int(0.5 + w * (1 << PRECISION_BITS))
    return K


def _pass(img: np.ndarray, K: np.ndarray, axis: int) -> np.ndarray:
    """One 8bpc pass along `axis` of an HWC uint8 image: clip8(sum(px * k) + 2^21 >> 22)."""
    x = img.astype(np.int64)
    if axis == 1:
        acc = np.einsum("hwc,ow->hoc", x, K)
    else:
        acc = np.einsum("hwc,oh->owc", x, K)
    acc = (acc + (1 << (PRECISION_BITS - 1))) >> PRECISION_BITS
    return np.clip(acc, 0, 255).astype(np.uint8)


def pil_resize_u8(img: np.ndarray, size) -> np.ndarray:
    """Image.resize((W_out, H_out), BICUBIC) of an RGB uint8 HWC array (ImagingResampleInner)."""
    H, W, _ = img.shape
    Ho, Wo = size
    out = img
    if Wo != W:  # need_horizontal
        out = _pass(out, precompute_coeffs(W, Wo), axis=1)
    if Ho != H:  # need_vertical
        out = _pass(out, precompute_coeffs(H, Ho), axis=0)
    return out.copy() if out is img else out


def center_crop_origin(size, crop):
    """torchvision center_crop: int(round((image - crop) / 2.0)) per axis."""
    return int(round((size[0] - crop[0]) / 2.0)), int(round((size[1] - crop[1]) / 2.0))


def val_transform(img: np.ndarray, image_size=(320, 320), crop_size=(224, 224), mean=IMAGENET_MEAN,
                  std=IMAGENET_STD):
    """(normalized fp32 CHW tensor, cropped uint8 HWC array) for one RGB uint8 HWC image."""
    r = pil_resize_u8(img, image_size)
    top, left = center_crop_origin(image_size, crop_size)
    u8 = r[top:top + crop_size[0], left:left + crop_size[1]]
    x = torch.from_numpy(np.ascontiguousarray(u8)).permute(2, 0, 1).to(torch.float32) / 255.0
    m = torch.tensor(mean, dtype=torch.float32)[:, None, None]
    s = torch.tensor(std, dtype=torch.float32)[:, None, None]
    return (x - m) / s, u8


def batch_metrics(logits: torch.Tensor, labels: torch.Tensor, num_classes: int, label_smoothing: float = 0.0):
    """(CE mean, BCE mean, correct count) of one batch as run_test computes them
    (model_test.py:69, :80-82; training_utilities.py:95-107)."""
    logits = logits.float()
    ce = F.cross_entropy(logits, labels)
    t = F.one_hot(labels, num_classes)
    t = t * (1 - label_smoothing) + label_smoothing / num_classes
    bce = F.binary_cross_entropy_with_logits(logits, t)
    correct = (logits.argmax(1) == labels).sum()
    return float(ce), float(bce), int(correct)
