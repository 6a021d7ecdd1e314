"""CPU oracle for the SdP-Net forward hot path — TEST INFRASTRUCTURE ONLY.

This module is a functional restatement of the reference forward pass
(y-akbal/SdP-Net @ 2025-06-14: model.py / layers.py / utility_layers.py /
training_utilities.py) written from its formulas in stock PyTorch CPU ops,
fp32.  It operates on a plain ``state_dict`` (same keys as the reference) and a
config dict (the 25 ``MainModel`` kwargs, model.py:28-54).

Who may use it: ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg, and only as the CHECKER / the timed CPU baseline.  The
product path (``sdp-net_amd/``) never imports it; the HIP path fails loudly when
its extension is missing.

Parity pinning: checked against golden logits produced by importing the
reference itself in the build container (``tests/golden/gen_golden.py``; the
reference ships no tests or golden vectors of its own).
Every function cites the reference file:line it restates.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor

# model.py:28-54 — MainModel constructor defaults.
MAINMODEL_DEFAULTS = dict(
    embedding_dim=128, num_blocks=10, n_head=4, activation="gelu",
    conv_kernel_size=5, patch_size=16, ffn_dropout=0.2, attn_dropout=0.2,
    output_classes=1000, conv_block_num=2, ff_multiplication_factor=4,
    max_image_size=[14, 14], max_num_registers=5, embedding_activation="none",
    conv_first=True, head_output_from_register=False, simple_mlp_output=False,
    output_head_bias=False, normalize_qv=True, stochastic_depth_p=[0.0, 0.0],
    mixer_deptwise_bias=False, mixer_ffn_bias=False, fast_att=True,
    conv_embedding=False, conv_embedding_kernel_size=5,
)


def full_config(cfg: dict) -> dict:
    out = dict(MAINMODEL_DEFAULTS)
    out.update(cfg)
    return out


# training_utilities.py:91-92
def kelu(x: Tensor, a: float = 3.5) -> Tensor:
    inner = 0.5 * x * (1 + x / a + (1 / math.pi) * torch.sin(x * math.pi / a))
    return torch.where(x < -a, torch.zeros_like(x), torch.where(x > a, x, inner))


# model.py:13-24 — activation registry ("fast_gelu" raises at forward in the
# reference: nn.GELU("fast") rejects the approximate string).
def activation(name: str, x: Tensor) -> Tensor:
    name = name.lower()
    if name == "gelu":
        return F.gelu(x)
    if name == "relu":
        return F.relu(x)
    if name == "tanh":
        return torch.tanh(x)
    if name == "sigmoid":
        return torch.sigmoid(x)
    if name == "leaky_relu":
        return F.leaky_relu(x, 0.01)
    if name == "selu":
        return F.selu(x)
    if name == "none":
        return x
    if name == "kelu":
        return kelu(x)
    raise ValueError(f"unknown activation {name}")


# layers.py:12-24 — channel LayerNorm on NCHW, biased variance, eps 1e-6,
# (var+eps)**0.5 division.
def channel_layernorm(x: Tensor, gamma: Tensor, beta: Tensor, eps: float = 1e-6) -> Tensor:
    mean = x.mean([1], keepdim=True)
    var = x.var([1], keepdim=True, unbiased=False)
    x = (x - mean) / (var + eps) ** 0.5
    return gamma[:, None, None] * x + beta[:, None, None]


# layers.py:40-42 — non-overlapping patch conv (stride = kernel = patch).
def conv_patcher(x: Tensor, sd: Dict[str, Tensor]) -> Tensor:
    w = sd["conv_init.conv.weight"]
    p = w.shape[-1]
    return F.conv2d(x, w, None, stride=p)


# layers.py:152-168 — x += Eh[:H]^T[:, :, None] + Ew[:W]^T[:, None, :];
# registers = Ereg[:num_registers+1] expanded over batch.
def embedding_layer(x: Tensor, sd: Dict[str, Tensor], num_registers: int,
                    act: str = "none") -> Tuple[Tensor, Tensor]:
    B, C, H, W = x.shape
    reg = sd["embedding_layer.register_embedding_layer.weight"][: num_registers + 1]
    # 'horizontal' table is indexed by H (rows), 'vertical' by W (columns): layers.py:158-159
    eh = sd["embedding_layer.horizontal_embedding_layer.weight"][:H].t().unsqueeze(-1)
    ew = sd["embedding_layer.vertical_embedding_layer.weight"][:W].t().unsqueeze(-2)
    x = x + eh
    x = x + ew
    return activation(act, x), reg.expand(B, reg.shape[-2], C)


# layers.py:202-209 — ConvEmbedding: x + AvgPool_k(bone); registers from
# Embedding[register buffer = 1..max_num_registers][:num_registers+1].
def conv_embedding_layer(x: Tensor, sd: Dict[str, Tensor], num_registers: int,
                         k: int, act: str = "none") -> Tuple[Tensor, Tensor]:
    B, C, H, W = x.shape
    bone = sd["embedding_layer.bone"]
    pos = F.avg_pool2d(bone[:, :, : H + k - 1, : W + k - 1], k, stride=1)
    idx = sd["embedding_layer.register"][: num_registers + 1].long()
    reg = sd["embedding_layer.register_embedding_layer.weight"][idx]
    return activation(act, x + pos), reg.expand(B, reg.shape[-2], C)


# layers.py:101-104 — ConvMixer (eval: drop paths are identity).
#   x_ = act(PW_CC(DW(LN1(x)))) + x ;  x = PW_down(act(PW_up(LN2(x_)))) + x_
def conv_mixer(x: Tensor, sd: Dict[str, Tensor], pre: str, act: str) -> Tensor:
    C = x.shape[1]
    dw_w = sd[pre + "conv2d.0.weight"]
    dw_b = sd.get(pre + "conv2d.0.bias")
    y = channel_layernorm(x, sd[pre + "layer_norm_1.gamma"], sd[pre + "layer_norm_1.beta"])
    y = F.conv2d(y, dw_w, dw_b, padding="same", groups=C)               # layers.py:73-78
    y = F.conv2d(y, sd[pre + "conv2d.1.weight"], sd.get(pre + "conv2d.1.bias"))  # :79-82
    x_ = activation(act, y) + x
    z = channel_layernorm(x_, sd[pre + "layer_norm_2.gamma"], sd[pre + "layer_norm_2.beta"])
    z = F.conv2d(z, sd[pre + "conv1d.0.weight"], sd.get(pre + "conv1d.0.bias"))  # :83-86
    z = activation(act, z)
    z = F.conv2d(z, sd[pre + "conv1d.2.weight"], sd.get(pre + "conv1d.2.bias"))  # :88-91
    return z + x_


# layers.py:259-316 — EncoderLayer in eval mode.
def encoder_layer(x: Tensor, reg: Tensor, sd: Dict[str, Tensor], pre: str, n_head: int,
                  act: str, normalize_qv: bool = True, fast_att: bool = True,
                  mask: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    B, C, H, W = x.shape
    R = reg.shape[1]
    hd = C // n_head
    t = torch.cat([reg, x.flatten(2).transpose(1, 2)], dim=1)          # :271-275
    h = F.layer_norm(t, (C,), sd[pre + "norm1.weight"], sd[pre + "norm1.bias"])  # :280
    q = F.linear(h, sd[pre + "q_proj.weight"]).view(B, R + H * W, n_head, hd).transpose(1, 2)
    k = F.linear(h, sd[pre + "k_proj.weight"]).view(B, R + H * W, n_head, hd).transpose(1, 2)
    v = F.linear(h, sd[pre + "v_proj.weight"]).view(B, R + H * W, n_head, hd).transpose(1, 2)
    if normalize_qv:                                                   # :236-237, :286
        q = F.layer_norm(q, (hd,), sd[pre + "q_norm.weight"], sd[pre + "q_norm.bias"])
        k = F.layer_norm(k, (hd,), sd[pre + "k_norm.weight"], sd[pre + "k_norm.bias"])
    if fast_att:                                                       # :289-291
        a = F.scaled_dot_product_attention(q, k, v, attn_mask=mask)
    else:                                                              # :292-298
        s = torch.matmul(q, k.transpose(-1, -2)) / (hd ** 0.5)
        if mask is not None:
            s = s.masked_fill(mask == 0, float("-inf"))
        a = torch.matmul(F.softmax(s, dim=-1), v)
    a = a.transpose(1, 2).contiguous().view(B, R + H * W, C)
    t = t + F.linear(a, sd[pre + "o_proj.weight"])                      # :301-303
    h = F.layer_norm(t, (C,), sd[pre + "norm2.weight"], sd[pre + "norm2.bias"])
    f = F.linear(h, sd[pre + "ff_linear1.weight"], sd[pre + "ff_linear1.bias"])
    f = F.linear(activation(act, f), sd[pre + "ff_linear2.weight"], sd[pre + "ff_linear2.bias"])
    t = t + f                                                          # :306-309
    reg, xf = t.split([R, H * W], dim=-2)                              # :311
    return xf.transpose(1, 2).reshape(B, C, H, W).contiguous(), reg     # :314


# layers.py:377-386
def block(x: Tensor, reg: Tensor, sd: Dict[str, Tensor], pre: str, cfg: dict,
          mask: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    act = cfg["activation"]

    def mixers(x):
        for j in range(cfg["conv_block_num"]):
            x = conv_mixer(x, sd, f"{pre}conv_blocks.{j}.", act)
        return x

    def enc(x, reg):
        return encoder_layer(x, reg, sd, pre + "t_block.", cfg["n_head"], act,
                             cfg["normalize_qv"], cfg["fast_att"], mask)

    if not cfg["conv_first"]:
        x, reg = enc(x, reg)
        return mixers(x), reg
    return enc(mixers(x), reg)


# layers.py:462-465 (+ head construction :443-460)
def classification_head(x: Tensor, reg: Tensor, sd: Dict[str, Tensor], cfg: dict) -> Tensor:
    p = "output_head.output_head."
    if cfg["head_output_from_register"]:
        h = reg.mean(-2)
        h = F.layer_norm(h, (h.shape[-1],), sd[p + "0.weight"], sd[p + "0.bias"])
        h = F.linear(h, sd[p + "1.weight"], sd.get(p + "1.bias"))
        if cfg["simple_mlp_output"]:
            return h
        h = torch.tanh(h)
        return F.linear(h, sd[p + "4.weight"], sd.get(p + "4.bias"))
    h = x.mean([-1, -2])
    return F.linear(h, sd[p + "2.weight"], sd.get(p + "2.bias"))


# model.py:129-149 — MainModel.forward (eval mode).
@torch.no_grad()
def forward(x: Tensor, sd: Dict[str, Tensor], cfg: dict, num_registers: int = 3,
            return_raw_outputs: bool = False):
    cfg = full_config(cfg)
    x = conv_patcher(x, sd)
    if cfg["conv_embedding"]:
        x, reg = conv_embedding_layer(x, sd, num_registers, cfg["conv_embedding_kernel_size"],
                                      cfg["embedding_activation"])
    else:
        x, reg = embedding_layer(x, sd, num_registers, cfg["embedding_activation"])
    for i in range(cfg["num_blocks"]):
        x, reg = block(x, reg, sd, f"blocks.{i}.", cfg)
    x, reg = encoder_layer(x, reg, sd, "final_block.t_block.", cfg["n_head"], cfg["activation"],
                           cfg["normalize_qv"], True)                  # FinalBlock: fast_att default
    logits = classification_head(x, reg, sd, cfg)
    if not return_raw_outputs:
        return logits
    return logits, x, reg
