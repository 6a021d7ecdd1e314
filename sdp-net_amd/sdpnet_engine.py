"""Host-side plumbing shared by the drop-in modules (layers.py / model.py).

* compute-dtype policy: bf16 when the input is bf16, the module's parameters are
  bf16, or a CUDA bf16 autocast region is active (the reference's "bf16 forward"
  is autocast, training_tools.py:85); fp32 otherwise.
* activation callables -> epilogue codes (model.py:13-24 registry, KeLu).
* per-module prepared-weight caches (bf16 casts, fused Wqkv, padded patch
  weight), keyed on the parameters' version counters so load_state_dict /
  optimizer steps invalidate them.  Not part of the state_dict.
"""
from __future__ import annotations

from typing import Callable, Dict, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

import sdpnet_hip as sp


def compute_dtype(x: torch.Tensor, module: nn.Module) -> torch.dtype:
    if not x.is_cuda:
        raise RuntimeError("sdpnet: the HIP forward needs CUDA (ROCm) tensors; there is no CPU fallback "
                           "(move the model and inputs with .to('cuda'))")
    if x.dtype == torch.float16:
        raise TypeError("sdpnet HIP path supports float32 and bfloat16 (not float16)")
    if torch.is_autocast_enabled("cuda"):
        ad = torch.get_autocast_dtype("cuda")
        if ad == torch.bfloat16:
            return torch.bfloat16
        raise TypeError(f"sdpnet HIP path supports bf16 autocast only, got {ad}")
    if x.dtype == torch.bfloat16:
        return torch.bfloat16
    for p in module.parameters():
        if p.dtype == torch.bfloat16:
            return torch.bfloat16
        break
    return torch.float32


def act_code(fn: Callable) -> int:
    """Map the reference's activation objects to epilogue codes."""
    if fn is None:
        return 0
    if isinstance(fn, nn.GELU):
        if fn.approximate != "none":
            # nn.GELU("fast") (model.py:16) raises at forward in the reference too.
            raise RuntimeError(f"approximate argument must be either none or tanh (got {fn.approximate!r}); "
                               "the HIP path implements exact-erf GELU only")
        return sp.ACT_CODES["gelu"]
    if fn is F.gelu:
        return sp.ACT_CODES["gelu"]
    if isinstance(fn, nn.ReLU) or fn is F.relu or fn is torch.relu:
        return sp.ACT_CODES["relu"]
    if isinstance(fn, nn.Tanh) or fn is torch.tanh:
        return sp.ACT_CODES["tanh"]
    if isinstance(fn, nn.Sigmoid) or fn is torch.sigmoid:
        return sp.ACT_CODES["sigmoid"]
    if isinstance(fn, nn.LeakyReLU):
        if abs(fn.negative_slope - 0.01) > 0:
            raise NotImplementedError("sdpnet HIP path implements LeakyReLU(0.01) only")
        return sp.ACT_CODES["leaky_relu"]
    if isinstance(fn, nn.SELU) or fn is F.selu:
        return sp.ACT_CODES["selu"]
    if isinstance(fn, nn.Identity):
        return sp.ACT_CODES["none"]
    if getattr(fn, "__name__", "") == "KeLu":
        return sp.ACT_CODES["kelu"]
    raise NotImplementedError(f"sdpnet HIP path: unsupported activation {fn!r}")


def _key(params, dtype, device):
    return (dtype, str(device)) + tuple((p._version, p.data_ptr()) for p in params)


def cached(module: nn.Module, name: str, params, dtype: torch.dtype, build: Callable[[], Dict]):
    """Return module._sdp_cache[name] rebuilt when any param changed."""
    cache = module.__dict__.setdefault("_sdp_cache", {})
    params = [p for p in params if p is not None]
    key = _key(params, dtype, params[0].device if params else "cpu")
    ent = cache.get(name)
    if ent is None or ent[0] != key:
        with torch.no_grad():
            ent = (key, build())
        cache[name] = ent
    return ent[1]


def as_dtype(t: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """Cast a parameter for the kernels (HIP cast kernel; no copy when already right)."""
    t = t.detach()
    if not t.is_contiguous():
        t = t.contiguous()
    if t.dtype == dtype:
        return t
    return sp.cast(t, dtype)


def f32(t):
    return None if t is None else as_dtype(t, torch.float32)


def num_reg_rows(max_num: int, num_registers: int) -> int:
    """Rows selected by `buffer[:num_registers+1]` (layers.py:157, :206)."""
    return len(range(max_num)[: num_registers + 1])


def hooked(module: nn.Module) -> bool:
    """True if any submodule has forward (pre-)hooks: the caller then composes
    the forward module by module so every hooked __call__ fires."""
    for m in module.modules():
        if m is module:
            continue
        if m._forward_hooks or m._forward_pre_hooks:
            return True
    return False
