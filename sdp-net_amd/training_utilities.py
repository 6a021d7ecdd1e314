"""Drop-in subset of ``training_utilities`` (reference training_utilities.py).

Provided: ``KeLu`` (training_utilities.py:91-92), the activation on the hot
path's activation registry (model.py:22), running on the HIP elementwise kernel
(the same code path the GEMM epilogues use), plus the two stateless helpers
``BCEWithLogitsLoss`` (:95-107) and ``MeasureTime`` (:118-132).

Not provided (out of scope): the wandb-logging loss/accuracy
trackers (:10-88).  This module does not import wandb.
"""
from __future__ import annotations

from typing import Callable

import torch

import sdpnet_hip as sp


def KeLu(x: torch.Tensor, a: float = 3.5) -> torch.Tensor:
    """0 for x < -a; x for x > a; 0.5 x (1 + x/a + sin(pi x / a) / pi) otherwise."""
    if a != 3.5:
        raise NotImplementedError("sdpnet HIP KeLu is compiled for a = 3.5 (the reference default)")
    if not x.is_cuda:
        raise RuntimeError("sdpnet KeLu runs on the HIP path only (CUDA/ROCm tensors)")
    xc = x.contiguous()
    if xc.dtype not in (torch.float32, torch.bfloat16):
        xc = xc.float()
    y = torch.empty_like(xc)
    sp.act(xc, y, sp.ACT_CODES["kelu"])
    return y


def BCEWithLogitsLoss(num_classes: int = 1000, label_smoothing: float = 0.1) -> Callable[[torch.Tensor, torch.Tensor], torch.Tensor]:
    def loss(input: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        if target.dim() == 1:
            target = torch.nn.functional.one_hot(target, num_classes)
        target_smoothed = target * (1 - label_smoothing) + label_smoothing / num_classes
        return torch.nn.functional.binary_cross_entropy_with_logits(input, target_smoothed)
    return loss


class MeasureTime:
    def __init__(self):
        self.start = torch.cuda.Event(enable_timing=True)
        self.stop = torch.cuda.Event(enable_timing=True)

    def __enter__(self):
        self.start.record()

    def __exit__(self, *args):
        self.stop.record()
        torch.cuda.synchronize()
        elapsed_time = self.start.elapsed_time(self.stop)
        print(f"Elapsed time: {elapsed_time/1000:.2f} seconds")
