"""On-device validation preprocessing.

Counterpart of the reference's ``val_transforms`` (hf_dataset_generator.py:27-41),
which ``model_test.py:50-52`` builds as ``val_transforms(image_size=(320, 320),
crop_size=(224, 224))``:

    RGB -> Resize(image_size, BICUBIC) -> CenterCrop(crop_size) -> ToImage
        -> ToDtype(float32, scale=True) -> Normalize(mean, std)

The reference applies it per PIL image on the dataloader's CPU workers.  Here a batch
of decoded images is packed into one pinned host buffer, copied once, and transformed
by ``sdp_val_preprocess`` (csrc/eval.hip) straight into the model's NCHW input, fp32 or
bf16.  The resize is Pillow's 8-bit resampler restated bit for bit (the crop's uint8
pixels equal PIL's), so images with an aspect ratio H / W above 100 -- where Pillow
changes its pass order -- are refused rather than approximated.
"""
from __future__ import annotations

import math
from typing import Iterable, List, Sequence, Tuple

import numpy as np
import torch

import sdpnet_hip as sp

IMAGENET_MEAN = (0.485, 0.456, 0.406)  # hf_dataset_generator.py:30-31
IMAGENET_STD = (0.229, 0.224, 0.225)
MAX_TAPS = 160


def _as_rgb_u8(img) -> np.ndarray:
    """transforms.RGB() + ToImage for one decoded image -> HWC uint8 (host)."""
    if hasattr(img, "convert") and hasattr(img, "mode"):  # PIL image
        if img.mode != "RGB":
            img = img.convert("RGB")
        return np.asarray(img, dtype=np.uint8)
    if isinstance(img, torch.Tensor):
        img = img.detach().cpu().numpy()
    a = np.asarray(img)
    if a.dtype != np.uint8:
        raise TypeError(f"val preprocessing takes decoded uint8 images, got {a.dtype}")
    if a.ndim == 2:
        a = np.repeat(a[:, :, None], 3, axis=2)
    if a.ndim != 3 or a.shape[2] not in (3, 4):
        raise ValueError(f"expected an HWC RGB image, got shape {a.shape}")
    return a[:, :, :3]


def _taps(n_in: int, n_out: int) -> int:
    return int(math.ceil(2.0 * max(1.0, n_in / n_out))) * 2 + 1


class ValTransform:
    """Batched ``val_transforms(image_size, crop_size, mean, std)``:
    ``__call__(images) -> Tensor[B, 3, crop_h, crop_w]`` on ``device``."""

    def __init__(self, image_size=(320, 320), crop_size=(224, 224), mean=IMAGENET_MEAN, std=IMAGENET_STD,
                 device="cuda", dtype=torch.float32):
        self.image_size = (int(image_size[0]), int(image_size[1]))
        self.crop_size = (int(crop_size[0]), int(crop_size[1]))
        if self.crop_size[0] > self.image_size[0] or self.crop_size[1] > self.image_size[1]:
            raise NotImplementedError("CenterCrop larger than the resized image (padding) is not supported")
        # torchvision center_crop origin: int(round((size - crop) / 2.0))
        self.top = int(round((self.image_size[0] - self.crop_size[0]) / 2.0))
        self.left = int(round((self.image_size[1] - self.crop_size[1]) / 2.0))
        self.mean, self.std = tuple(mean), tuple(std)
        self.device = torch.device(device)
        self.dtype = dtype

    def __call__(self, images: Sequence, return_u8: bool = False):
        arrs = [_as_rgb_u8(im) for im in images]
        B = len(arrs)
        RH, RW = self.image_size
        if B == 0:
            out = torch.empty(0, 3, *self.crop_size, dtype=self.dtype, device=self.device)
            u8 = torch.empty(0, *self.crop_size, 3, dtype=torch.uint8, device=self.device)
            return (out, u8) if return_u8 else out
        kmax, hmax, wmax = 1, 1, 1
        for a in arrs:
            H, W = a.shape[:2]
            if H == 0 or W == 0:
                raise ValueError("empty image")
            if H > 100 * W:
                raise NotImplementedError(f"image {H}x{W}: aspect ratio above 100 (Pillow reorders its passes there)")
            kmax = max(kmax, _taps(W, RW), _taps(H, RH))
            hmax = max(hmax, H)
            wmax = max(wmax, W)
        if kmax > MAX_TAPS:
            raise NotImplementedError(f"downscale factor too large ({kmax} taps > {MAX_TAPS})")
        sizes = [a.shape[0] * a.shape[1] * 3 for a in arrs]
        offs = np.zeros(B, dtype=np.int64)
        offs[1:] = np.cumsum(sizes)[:-1]
        host = torch.empty(sum(sizes), dtype=torch.uint8, pin_memory=torch.cuda.is_available())
        hv = host.numpy()
        for a, o, n in zip(arrs, offs, sizes):
            hv[o:o + n] = np.ascontiguousarray(a).reshape(-1)
        hw = torch.tensor([[a.shape[0], a.shape[1]] for a in arrs], dtype=torch.int32)
        pix = host.to(self.device, non_blocking=True)
        offs_d = torch.from_numpy(offs).to(self.device)
        hw_d = hw.to(self.device)
        tmp_stride = hmax * self.crop_size[1] * 4  # RGBX words of the horizontal pass
        out, u8 = sp.val_preprocess(pix, offs_d, hw_d, self.image_size, self.crop_size, self.top, self.left, kmax,
                                    self.mean, self.std, tmp_stride, self.dtype, want_u8=return_u8, max_w=wmax)
        return (out, u8) if return_u8 else out


def val_transforms(image_size=(320, 320), crop_size=(224, 224), mean=IMAGENET_MEAN, std=IMAGENET_STD,
                   device="cuda", dtype=torch.float32) -> ValTransform:
    """hf_dataset_generator.py:27-41 signature; returns the batched device transform."""
    return ValTransform(image_size, crop_size, mean, std, device=device, dtype=dtype)


def batches(dataset: Iterable, transform: ValTransform, batch_size: int = 256) -> Iterable[Tuple[torch.Tensor, torch.Tensor]]:
    """(images, labels) device batches from an iterable of (decoded image, int label)
    pairs -- the hf_dataset + DataLoader(batch_size=256, shuffle=False) of
    model_test.py:52-53 with the transform moved onto the GPU."""
    imgs: List = []
    labels: List[int] = []
    for img, lab in dataset:
        imgs.append(img)
        labels.append(int(lab))
        if len(imgs) == batch_size:
            yield transform(imgs), torch.tensor(labels, dtype=torch.int64).to(transform.device)
            imgs, labels = [], []
    if imgs:
        yield transform(imgs), torch.tensor(labels, dtype=torch.int64).to(transform.device)
