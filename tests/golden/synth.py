"""Deterministic, portable synthetic weights and inputs (test infrastructure).

The reference ships no checkpoints, so parity is pinned on weights that the
build generates itself, identically here (where the reference is imported to
make the golden logits) and on the GPU box (where the reference does not exist).

PRNG: splitmix64 counter stream (seeded per tensor by crc32 of its state_dict
key), uniform from the top 53 bits, Box-Muller for normals.  Pure numpy, no
version-dependent distribution code.

Init distributions follow the reference (model.py:121-126):
  * every Linear / Conv2d weight: trunc_normal(std=0.01, a=-2, b=2)
  * Linear / Conv2d biases: U(-1/sqrt(fan_in), 1/sqrt(fan_in)) (torch default)
  * nn.Embedding: N(0, 1)
  * LayerNorm affine: the reference starts at gamma=1, beta=0; here gamma is
    perturbed to 1 + 0.05 N and beta to 0.05 N so that an affine bug shows up.
  * ConvEmbedding 'bone' buffer: 0.02 N (layers.py:194-197)
  * integer index buffers: arange (as constructed).
"""
from __future__ import annotations

import zlib
from typing import Dict

import numpy as np
import torch

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(seed: int, n: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
             + np.uint64(seed & 0xFFFFFFFFFFFFFFFF))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(seed: int, n: int) -> np.ndarray:
    """U[0,1) float64, strictly > 0."""
    z = _splitmix64(seed, n)
    return ((z >> np.uint64(11)).astype(np.float64) + 0.5) * (1.0 / 9007199254740992.0)


def normal(seed: int, n: int) -> np.ndarray:
    m = (n + 1) // 2
    u = uniform(seed, 2 * m)
    u1, u2 = u[:m], u[m:]
    r = np.sqrt(-2.0 * np.log(u1))
    out = np.empty(2 * m, dtype=np.float64)
    out[0::2] = r * np.cos(2 * np.pi * u2)
    out[1::2] = r * np.sin(2 * np.pi * u2)
    return out[:n]


def key_seed(seed: int, key: str) -> int:
    return (seed * 0x100000001B3 + zlib.crc32(key.encode())) & 0xFFFFFFFFFFFFFFFF


def synth_tensor(seed: int, key: str, shape, kind: str, fan_in: int = 1) -> torch.Tensor:
    n = int(np.prod(shape)) if len(shape) else 1
    s = key_seed(seed, key)
    if kind == "w":
        v = np.clip(normal(s, n) * 0.01, -2.0, 2.0)
    elif kind == "b":
        bound = 1.0 / np.sqrt(fan_in)
        v = (uniform(s, n) * 2.0 - 1.0) * bound
    elif kind == "emb":
        v = normal(s, n)
    elif kind == "gamma":
        v = 1.0 + 0.05 * normal(s, n)
    elif kind == "beta":
        v = 0.05 * normal(s, n)
    elif kind == "bone":
        v = 0.02 * normal(s, n)
    else:
        raise ValueError(kind)
    return torch.from_numpy(v.astype(np.float32).reshape(shape))


def synth_state_dict(model: torch.nn.Module, seed: int) -> Dict[str, torch.Tensor]:
    """Build a state_dict for ``model`` (the reference's or ours: both have the
    same module tree) from the portable PRNG.  Module types are recognised by
    class name so the same code serves both implementations."""
    out: Dict[str, torch.Tensor] = {}
    for mname, mod in model.named_modules():
        cls = mod.__class__.__name__
        pre = mname + "." if mname else ""
        for pname, p in mod.named_parameters(recurse=False):
            key = pre + pname
            shape = tuple(p.shape)
            if cls in ("Linear", "Conv2d"):
                if pname == "weight":
                    out[key] = synth_tensor(seed, key, shape, "w")
                else:
                    w = getattr(mod, "weight")
                    fan_in = int(np.prod(w.shape[1:]))
                    out[key] = synth_tensor(seed, key, shape, "b", fan_in)
            elif cls == "Embedding":
                out[key] = synth_tensor(seed, key, shape, "emb")
            elif cls == "LayerNorm":
                kind = "gamma" if pname in ("weight", "gamma") else "beta"
                out[key] = synth_tensor(seed, key, shape, kind)
            elif pname == "bone":
                out[key] = synth_tensor(seed, key, shape, "bone")
            else:
                raise ValueError(f"no synth rule for {key} ({cls})")
        for bname, b in mod.named_buffers(recurse=False):
            key = pre + bname
            if bname == "bone":
                out[key] = synth_tensor(seed, key, tuple(b.shape), "bone")
            else:
                out[key] = b.detach().clone()
    sd = model.state_dict()
    assert list(out.keys()) == [k for k in sd.keys() if k in out] and set(out) == set(sd), \
        "synth_state_dict did not cover the model's state_dict"
    return {k: out[k] for k in sd.keys()}


def synth_images(seed: int, batch: int, size: int = 224) -> torch.Tensor:
    n = batch * 3 * size * size
    return torch.from_numpy(normal(key_seed(seed, "images"), n).astype(np.float32)
                            .reshape(batch, 3, size, size))


# Canonical configurations: model_config_vit.yaml:9-33 + overrides.
YAML_BASE = dict(
    embedding_dim=768, num_blocks=6, n_head=8, activation="gelu", embedding_activation="none",
    conv_kernel_size=3, patch_size=14, ffn_dropout=0.2, attn_dropout=0.2, output_classes=1000,
    conv_block_num=2, ff_multiplication_factor=4, max_image_size=[16, 16], max_num_registers=5,
    conv_first=False, head_output_from_register=True, simple_mlp_output=False,
    output_head_bias=False, normalize_qv=True, stochastic_depth_p=[0.0, 0.0],
    mixer_deptwise_bias=False, mixer_ffn_bias=False, conv_embedding=False,
    conv_embedding_kernel_size=5,
)


def canonical(name: str, **over) -> dict:
    sizes = {
        "XXS": dict(embedding_dim=128, num_blocks=7, patch_size=16, conv_kernel_size=7),
        "M": dict(embedding_dim=768, num_blocks=12, patch_size=16, conv_kernel_size=7),
        "XL": dict(embedding_dim=768, num_blocks=17, patch_size=14, conv_kernel_size=7),
    }
    cfg = dict(YAML_BASE)
    cfg.update(sizes[name])
    cfg["conv_first"] = True  # measure with conv_first=True; parity-test both
    cfg.update(over)
    return cfg
