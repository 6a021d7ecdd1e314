"""Checkpoint / evaluation harness on the HIP path.

Counterpart of the reference's ``model_test.py`` (same function names and loop), named
``eval_harness`` so test collectors do not mistake it for a test module:

* ``preprocess_weights`` (model_test.py:21-26): strip the DDP ``"module."`` prefix --
  and the ``torch.compile`` ``"_orig_mod."`` prefix a compiled model's state_dict
  carries -- and move tensors to the CPU.
* ``return_model`` (:28-42): a training checkpoint ``{"model_config",
  "model_state_dict", ...}`` (training_tools.py:203-221) and an EMA weights file (a
  plain state_dict, training_tools.py:300-302) -> (model, ema_model) in eval mode.
  Files are read with ``torch.load(weights_only=True)``: nothing in them executes.
* ``return_dataloader`` (:44-54): device batches through the on-device validation
  transform (preprocess.py).  ImageNet itself needs the network, so the caller passes
  the (decoded image, label) pairs.
* ``run_test`` (:58-85): the same running CE / BCE / accuracy loop and print line, with
  the per-row metrics computed by ``sdp_logits_metrics`` (csrc/eval.hip).
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, Optional, Tuple

import torch

import sdpnet_hip as sp
from model import MainModel
from preprocess import batches, val_transforms

MODEL_DIR = "."
MODEL_WEIGHTS_NAME = "model_1_cp281.pt"   # model_test.py:12-13
EMA_WEIGHTS_NAME = "ema_model_cp281.pt"
DEVICE = "cuda"                           # the HIP path has no CPU device
COMPILE_MODEL = True                      # model_test.py:16
PREFIXES = ("module.", "_orig_mod.")


def preprocess_weights(weights: dict, excluded_key="module.") -> Dict[str, torch.Tensor]:
    """model_test.py:21-26 (plus the torch.compile prefix)."""
    keys = (excluded_key,) if isinstance(excluded_key, str) else tuple(excluded_key)
    keys = keys + tuple(p for p in PREFIXES if p not in keys)
    new_weights = {}
    for key, value in weights.items():
        k = key
        for p in keys:
            k = k.replace(p, "")
        new_weights[k] = value.to("cpu") if isinstance(value, torch.Tensor) else value
    return new_weights


def _load(path: str):
    return torch.load(path, map_location="cpu", weights_only=True)


def return_model(model_path: str = MODEL_DIR, model_weights_name: str = MODEL_WEIGHTS_NAME,
                 ema_weights_name: Optional[str] = EMA_WEIGHTS_NAME) -> Tuple[MainModel, Optional[MainModel]]:
    """model_test.py:28-42: (model, ema_model), both eval-mode on the CPU."""
    weights = _load(os.path.join(model_path, model_weights_name))
    model = MainModel.from_dict(**weights["model_config"])
    model.load_state_dict(preprocess_weights(weights["model_state_dict"]))
    model.eval()
    ema_model = None
    if ema_weights_name is not None:
        ema_weights = _load(os.path.join(model_path, ema_weights_name))
        ema_model = MainModel.from_dict(**weights["model_config"])
        ema_model.load_state_dict(preprocess_weights(ema_weights))
        ema_model.eval()
    return model, ema_model


def return_dataloader(dataset: Iterable, batch_size: int = 256, image_size=(320, 320), crop_size=(224, 224),
                      device=DEVICE, dtype=torch.float32):
    """model_test.py:44-54 with the transform on the GPU: yields (images, labels) on device."""
    return batches(dataset, val_transforms(image_size, crop_size, device=device, dtype=dtype), batch_size)


def batch_metrics(outputs: torch.Tensor, labels: torch.Tensor, num_classes: int, label_smoothing: float = 0.0):
    """(mean CE, mean BCE, correct) of one batch (model_test.py:80-82) from sdp_logits_metrics."""
    if outputs.shape[1] != num_classes:
        raise ValueError(f"logits have {outputs.shape[1]} classes, expected {num_classes}")
    m = sp.logits_metrics(outputs.contiguous(), labels.to(torch.int64), label_smoothing)
    B = outputs.shape[0]
    s = m.sum(0).tolist()  # one device -> host sync per batch, as the reference's .item()s
    return s[0] / B, s[1] / (B * num_classes), int(s[2])


def run_test(model: Optional[MainModel] = None, ema_model: Optional[MainModel] = None,
             test_data: Optional[Iterable] = None, compile_model: bool = COMPILE_MODEL, num_classes: int = 1000,
             verbose: bool = True) -> Dict[str, float]:
    """model_test.py:58-85.  Returns the final {CrossEntropyLoss, BCEWithLogitsLoss,
    Accuracy}; like the reference, only ``model`` is scored (``ema_model`` is moved and
    compiled alongside it)."""
    if model is None:
        model, ema_model = return_model()
    if test_data is None:
        raise ValueError("pass test_data: ImageNet (model_test.py:45) needs the network")
    model = model.to(DEVICE).eval()
    if ema_model is not None:
        ema_model = ema_model.to(DEVICE).eval()
    if compile_model:
        model = torch.compile(model)
        ema_model = torch.compile(ema_model) if ema_model is not None else None
    temp_loss_1, temp_loss_2, acc, size, num_batch = 0.0, 0.0, 0, 0, 0
    for images, labels in test_data:
        images, labels = images.to(DEVICE), labels.to(DEVICE)
        with torch.no_grad():
            outputs = model(images)
            ce, bce, correct = batch_metrics(outputs, labels, num_classes)
            temp_loss_1 += ce
            temp_loss_2 += bce
            acc += correct
            size += len(labels)
            num_batch += 1
        if verbose:
            print(f"CrossEntropyLoss: {temp_loss_1/num_batch}, BCEWithLogitsLoss: {temp_loss_2/num_batch}, "
                  f"Accuracy: {acc/size}")
    if num_batch == 0:
        return {"CrossEntropyLoss": float("nan"), "BCEWithLogitsLoss": float("nan"), "Accuracy": float("nan")}
    return {"CrossEntropyLoss": temp_loss_1 / num_batch, "BCEWithLogitsLoss": temp_loss_2 / num_batch,
            "Accuracy": acc / size}


if __name__ == "__main__":
    run_test()
