"""Drop-in ``layers`` module: the reference's block classes (layers.py of
y-akbal/SdP-Net @ 2025-06-14) with the same names, constructor arguments,
module trees / state_dict keys and forward signatures, whose forwards run on the
gfx950 HIP kernels of libsdpnet_hip.so (no ATen compute, no CPU fallback).

Layout.  Internally every block works on a token-major buffer [B, R+HW, C]
(registers first, layers.py:275) so the NCHW<->token flatten/concat/split of the
reference (layers.py:271-275, :311-314) disappears on the fused MainModel path.
The standalone NCHW forwards below convert at entry/exit with HIP transpose
kernels and share the token-level ``_run_*`` code with the fused path.

Module construction mirrors the reference order exactly, so the same
``torch.manual_seed`` yields bit-identical initial parameters.
"""
from __future__ import annotations

import os
from typing import Callable, Optional, Tuple

import torch
from torch import nn as nn
from torch.nn import functional as F
from torch.nn.parameter import Parameter

import sdpnet_hip as sp
from sdpnet_engine import (act_code, as_dtype, cached, compute_dtype, f32, hooked, num_reg_rows)
from utility_layers import StochasticDepth as SD


def _train():
    """sdpnet_train, imported at call time (train-mode forwards of the sub-modules)."""
    import sdpnet_train
    return sdpnet_train


Rows = sp.Rows


def _dense(t: torch.Tensor) -> Rows:
    return Rows(t, t.shape[-1])


# A/B switch (benchmarks): SDPNET_LN_FOLD=0 runs the LayerNorms as separate row-LN
# kernels feeding unfolded GEMMs (the statistics still come from the partials).
_LN_FOLD = os.environ.get("SDPNET_LN_FOLD", "1") != "0"


def new_partials(rows: int, C: int, device) -> torch.Tensor:
    """LayerNorm statistics by parts of a token buffer: [rows, ceil(C/64), 2] fp32
    {mean, M2} per 64-column chunk of each physical row (sdp_row_partials /
    sdp_gemm_ln write them, sdp_ln_stats combines them)."""
    return torch.empty(rows, (C + 63) // 64, 2, dtype=torch.float32, device=device)


def _ln_stats(part: torch.Tensor, rows: Rows, M: int, C: int, eps: float) -> torch.Tensor:
    st = torch.empty(M, 2, dtype=torch.float32, device=part.device)
    sp.ln_stats(part, rows, M, C, eps, st)
    return st


def _fold(w: torch.Tensor, ln: nn.Module, bias: Optional[torch.Tensor], dt):
    """(W*gamma in dt, colsum, beta.W^T + b) of a Linear consuming LN(x)."""
    g = ln.gamma if hasattr(ln, "gamma") else ln.weight
    b = ln.beta if hasattr(ln, "beta") else ln.bias
    return sp.fold_ln_weight(f32(w), f32(g), f32(b), f32(bias), dt)


class LayerNorm(nn.Module):
    """Channel LayerNorm over dim 1 of NCHW, biased variance, eps 1e-6
    (layers.py:12-24).  On the token layout it is a row LN over C."""

    def __init__(self, embedding_dim: int, eps: float = 1e-6):
        super().__init__()
        self.gamma = nn.Parameter(torch.ones(embedding_dim))
        self.beta = nn.Parameter(torch.zeros(embedding_dim))
        self.eps = eps

    def _params(self):
        return cached(self, "ln", [self.gamma, self.beta], torch.float32,
                      lambda: (f32(self.gamma), f32(self.beta)))

    def _run_rows(self, x: Rows, y: Rows, M: int):
        g, b = self._params()
        sp.layernorm(x, g, b, self.eps, y, M, self.gamma.shape[0])

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.training:
            return _train().train_layernorm(self, x)
        dt = compute_dtype(x, self)
        with torch.no_grad():
            x = x.to(dt).contiguous()
            B, C, H, W = x.shape
            rows = torch.empty(B * H * W, C, dtype=dt, device=x.device)
            sp.nchw_to_rows(x, _dense(rows))
            self._run_rows(_dense(rows), _dense(rows), B * H * W)
            out = torch.empty_like(x)
            sp.rows_to_nchw(_dense(rows), out)
            return out


class ConvPatcher(nn.Module):
    """Patch embedding Conv2d(3, C, k=s=p, no bias) (layers.py:28-42) as
    im2col + MFMA GEMM."""

    def __init__(self, embedding_dim=128, patch_size=4):
        super().__init__()
        self.conv = nn.Conv2d(in_channels=3, out_channels=embedding_dim, kernel_size=patch_size,
                              stride=patch_size, bias=False)

    @property
    def patch_size(self) -> int:
        return self.conv.kernel_size[0]

    def _kpad(self) -> int:
        k = 3 * self.patch_size ** 2
        return (k + 63) // 64 * 64

    def _weight(self, dt):
        def build():
            C = self.conv.out_channels
            w = as_dtype(self.conv.weight.reshape(C, -1), dt)
            kp = self._kpad()
            if kp == w.shape[1]:
                return w
            wp = torch.zeros(C, kp, dtype=dt, device=w.device)
            wp[:, : w.shape[1]].copy_(w)
            return wp
        return cached(self, "w", [self.conv.weight], dt, build)

    def _run(self, img: torch.Tensor, dt, y: Rows, resid: Optional[Rows] = None, act: int = 0,
             part: Optional[torch.Tensor] = None):
        """img [B,3,Hi,Wi] -> y rows (logical row = b*P + ph*Wp + pw); ``part``: token
        LN partial statistics the output rows' are written to."""
        B, _, Hi, Wi = img.shape
        p = self.patch_size
        P = (Hi // p) * (Wi // p)
        kp = self._kpad()
        patches = torch.empty(B * P, kp, dtype=dt, device=img.device)
        sp.patchify(img.contiguous(), patches, p, kp)
        w = self._weight(dt)
        sp.gemm(_dense(patches), w, y, B * P, w.shape[0], kp, resid=resid, act=act, resid_pre=True, part=part)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.training:
            return _train().train_patcher(self, x)
        dt = compute_dtype(x, self)
        with torch.no_grad():
            B, _, Hi, Wi = x.shape
            p = self.patch_size
            Hp, Wp = Hi // p, Wi // p
            C = self.conv.out_channels
            rows = torch.empty(B * Hp * Wp, C, dtype=dt, device=x.device)
            self._run(x, dt, _dense(rows))
            out = torch.empty(B, C, Hp, Wp, dtype=dt, device=x.device)
            sp.rows_to_nchw(_dense(rows), out)
            return out


class ConvMixer(nn.Module):
    """x_ = act(PW_CC(DW_k(LN1(x)))) + x ;  x = PW_down(act(PW_up(LN2(x_)))) + x_
    (layers.py:63-104).  Hidden width is hard-coded 4C (layers.py:84, :88)."""

    def __init__(self, embedding_dim: int = 768, kernel_size: int = 5, activation: Callable = nn.GELU(),
                 drop_p: float = 0.0, mixer_ffn_bias: bool = True, mixer_deptwise_bias: bool = True):
        super().__init__()
        self.conv2d = nn.Sequential(*[
            nn.Conv2d(in_channels=embedding_dim, out_channels=embedding_dim, kernel_size=kernel_size,
                      groups=embedding_dim, padding="same", bias=mixer_deptwise_bias),
            nn.Conv2d(in_channels=embedding_dim, out_channels=embedding_dim, kernel_size=1, bias=mixer_ffn_bias)])
        self.conv1d = nn.Sequential(*[
            nn.Conv2d(in_channels=embedding_dim, out_channels=4 * embedding_dim, kernel_size=1, bias=mixer_ffn_bias),
            activation,
            nn.Conv2d(in_channels=4 * embedding_dim, out_channels=embedding_dim, kernel_size=1, bias=mixer_ffn_bias)])
        self.layer_norm_1 = LayerNorm(embedding_dim)
        self.layer_norm_2 = LayerNorm(embedding_dim)
        self.activation = activation
        self.drop_path_1 = SD(drop_p) if drop_p > 1e-5 else nn.Identity()
        self.drop_path_2 = SD(drop_p) if drop_p > 1e-5 else nn.Identity()

    def _prep(self, dt):
        dw, cc, up, dn = self.conv2d[0], self.conv2d[1], self.conv1d[0], self.conv1d[2]
        ln2 = self.layer_norm_2
        params = [dw.weight, dw.bias, cc.weight, cc.bias, up.weight, up.bias, dn.weight, dn.bias,
                  ln2.gamma, ln2.beta]

        def build():
            C = cc.out_channels
            # layer_norm_2 folded into the up projection (sdp_gemm_ln)
            up_w, up_s, up_c = _fold(up.weight.reshape(4 * C, C), ln2, up.bias, dt)
            if not _LN_FOLD:
                up_w, up_s, up_c = as_dtype(up.weight.reshape(4 * C, C), dt), None, f32(up.bias)
            return dict(
                k=dw.kernel_size[0],
                dw_w=f32(dw.weight.reshape(C, -1)), dw_b=f32(dw.bias),
                cc_w=as_dtype(cc.weight.reshape(C, C), dt), cc_b=f32(cc.bias),
                up_w=up_w, up_s=up_s, up_c=up_c,
                dn_w=as_dtype(dn.weight.reshape(C, 4 * C), dt), dn_b=f32(dn.bias))
        return cached(self, "w", params, dt, build)

    def _run_tokens(self, img: Rows, B: int, H: int, W: int, dt, part: Optional[torch.Tensor] = None):
        """In-place on the image rows ``img`` (logical row b*H*W + h*W + w).  ``part``:
        the token buffer's LN partial statistics (current for these rows; kept
        current on return); computed here when not given."""
        C = self.conv2d[1].out_channels
        M = B * H * W
        w = self._prep(dt)
        a = act_code(self.activation)
        dev = img.t.device
        if part is None:
            part = new_partials(img.t.shape[0], C, dev)
            sp.row_partials(img, M, C, part)
        # LN1 fused into the depthwise conv: (mean, rstd) from the partials, normalise-on-load (layers.py:102)
        stats = _ln_stats(part, img, M, C, self.layer_norm_1.eps)
        g1, b1 = self.layer_norm_1._params()
        dwo = torch.empty(M, C, dtype=dt, device=dev)
        sp.dwconv(img, w["dw_w"], w["dw_b"], _dense(dwo), B, H, W, C, w["k"], stats=stats, ln_gamma=g1, ln_beta=b1)
        # x_ = act(PW(DW(LN1 x)) + b) + x      (layers.py:102); emits x_'s LN partials
        sp.gemm(_dense(dwo), w["cc_w"], img, M, C, C, bias=w["cc_b"], resid=img, act=a, part=part)
        # hid = act(PW_up(LN2 x_) + b) with LN2 folded into the GEMM (layers.py:103)
        hid = torch.empty(M, 4 * C, dtype=dt, device=dev)
        if _LN_FOLD:
            stats2 = _ln_stats(part, img, M, C, self.layer_norm_2.eps)
            sp.gemm(img, w["up_w"], _dense(hid), M, 4 * C, C, bias=w["up_c"], act=a, ln=(stats2, w["up_s"]))
        else:
            ln = torch.empty(M, C, dtype=dt, device=dev)
            self.layer_norm_2._run_rows(img, _dense(ln), M)
            sp.gemm(_dense(ln), w["up_w"], _dense(hid), M, 4 * C, C, bias=w["up_c"], act=a)
        # x = PW_down(hid) + b + x_             (layers.py:103); emits x's LN partials
        sp.gemm(_dense(hid), w["dn_w"], img, M, C, 4 * C, bias=w["dn_b"], resid=img, part=part)

    def forward(self, x: torch.Tensor):
        if self.training:
            return _train().train_conv_mixer(self, x)
        dt = compute_dtype(x, self)
        with torch.no_grad():
            x = x.to(dt).contiguous()
            B, C, H, W = x.shape
            rows = torch.empty(B * H * W, C, dtype=dt, device=x.device)
            sp.nchw_to_rows(x, _dense(rows))
            self._run_tokens(_dense(rows), B, H, W, dt)
            out = torch.empty_like(x)
            sp.rows_to_nchw(_dense(rows), out)
            return out


class EmbeddingLayer(nn.Module):
    """Row/column positional embeddings + register tokens (layers.py:116-168).
    The 'horizontal' table is indexed by H (rows), the 'vertical' one by W."""

    def __init__(self, embedding_dim: int = 768, max_num_registers: int = 5, max_image_size: list = [14, 14],
                 activation: Callable = None):
        super().__init__()
        self.max_num_registers = max_num_registers
        self.activation = activation if activation != None else torch.nn.Identity()  # noqa: E711
        self.register_embedding_layer = nn.Embedding(max_num_registers, embedding_dim)
        self.vertical_embedding_layer = nn.Embedding(max_image_size[0], embedding_dim)
        self.horizontal_embedding_layer = nn.Embedding(max_image_size[1], embedding_dim)
        self.register_buffer("register_embeddings", torch.arange(max_num_registers, dtype=torch.int))
        self.register_buffer("vertical_embedding", torch.arange(max_image_size[0], dtype=torch.int))
        self.register_buffer("horizontal_embedding", torch.arange(max_image_size[1], dtype=torch.int))

    def _pos_table(self, H: int, W: int) -> torch.Tensor:
        """fp32 [H*W, C]: Eh[h] + Ew[w] (layers.py:158-163)."""
        eh = self.horizontal_embedding_layer.weight
        ew = self.vertical_embedding_layer.weight
        if H > eh.shape[0] or W > ew.shape[0]:
            # the reference fails to broadcast in the same situation
            raise RuntimeError(f"image grid {H}x{W} exceeds max_image_size {[ew.shape[0], eh.shape[0]]}")
        C = eh.shape[1]
        def build():
            t = torch.empty(H * W, C, dtype=torch.float32, device=eh.device)
            sp.pos_table(f32(eh), f32(ew), t, H, W, C)
            return t
        return cached(self, f"pos{H}x{W}", [eh, ew], torch.float32, build)

    def _register_rows(self, num_registers: int) -> Tuple[torch.Tensor, int]:
        """(table fp32 [>=R, C] whose first R rows are the registers, R)."""
        R = num_reg_rows(self.max_num_registers, num_registers)
        return f32(self.register_embedding_layer.weight), R

    def forward(self, x: torch.Tensor, num_registers: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
        if self.training:
            return _train().train_pos_embedding(self, x, num_registers)
        dt = compute_dtype(x, self)
        with torch.no_grad():
            B, C, H, W = x.shape
            if x.dtype != dt or not x.is_contiguous():
                x = x.to(dt).contiguous()
            sp.nchw_add_table(x, self._pos_table(H, W))          # x += ... in place (layers.py:162-163)
            code = act_code(self.activation)
            out = x
            if code != 0:
                out = torch.empty_like(x)
                sp.act(x, out, code)
            table, R = self._register_rows(num_registers)
            regs = torch.empty(B, R, C, dtype=dt, device=x.device)
            sp.copy_rows(table, C, 0, regs, C, R * C, B, R, C)
            return out, regs


class ConvEmbedding(nn.Module):
    """x + AvgPool_k(bone) positional embedding + registers from
    Embedding[1..R] (layers.py:174-209).  Note the reference re-seeds the global
    RNG in __init__ (layers.py:185); mirrored."""

    def __init__(self, embedding_dim: int = 768, kernel_size: int = 5, activation: Callable = nn.GELU(),
                 max_image_size: list = [14, 14], max_num_registers: int = 5, seed: int = 0,
                 trainable_bone: bool = False):
        super().__init__()
        torch.manual_seed(seed)
        self.conv2d = nn.AvgPool2d(kernel_size, stride=1)
        self.kernel_size = kernel_size
        if trainable_bone:
            self.register_parameter("bone", Parameter(0.02 * torch.randn(1, embedding_dim,
                                                                         max_image_size[0] + kernel_size,
                                                                         max_image_size[1] + kernel_size)))
        else:
            self.register_buffer("bone", 0.02 * torch.randn(1, embedding_dim, max_image_size[0] + kernel_size,
                                                            max_image_size[1] + kernel_size, requires_grad=False))
        self.register_buffer("register", torch.arange(1, max_num_registers + 1, dtype=torch.int))
        self.register_embedding_layer = nn.Embedding(max_num_registers, embedding_dim)
        self.activation = activation if activation != None else torch.nn.Identity()  # noqa: E711

    def _pos_table(self, H: int, W: int) -> torch.Tensor:
        bone = self.bone
        C = bone.shape[1]
        k = self.kernel_size
        def build():
            t = torch.empty(H * W, C, dtype=torch.float32, device=bone.device)
            sp.avgpool_table(f32(bone), t, H, W, C, k)
            return t
        return cached(self, f"pos{H}x{W}", [bone], torch.float32, build)

    def _register_rows(self, num_registers: int) -> Tuple[torch.Tensor, int]:
        # rows register[:num_registers+1] = 1..R of the embedding table (layers.py:206)
        R = num_reg_rows(self.register.shape[0], num_registers)
        idx = self.register[:R].long()
        w = self.register_embedding_layer.weight
        if R > 0 and (int(idx[-1]) >= w.shape[0]):
            raise IndexError("index out of range in self")  # nn.Embedding's error (layers.py:206)
        t = f32(w)
        return t[1:] if R > 0 else t, R

    def forward(self, x: torch.Tensor, num_registers: int = 3) -> Tuple[torch.Tensor, torch.Tensor]:
        if self.training:
            return _train().train_pos_embedding(self, x, num_registers)
        dt = compute_dtype(x, self)
        with torch.no_grad():
            B, C, H, W = x.shape
            xx = x.to(dt).contiguous().clone()
            sp.nchw_add_table(xx, self._pos_table(H, W))
            code = act_code(self.activation)
            if code != 0:
                sp.act(xx, xx, code)
            table, R = self._register_rows(num_registers)
            regs = torch.empty(B, R, C, dtype=dt, device=x.device)
            sp.copy_rows(table.contiguous(), C, 0, regs, C, R * C, B, R, C)
            return xx, regs


class EncoderLayer(nn.Module):
    """Pre-LN transformer encoder over [registers; image tokens]
    (layers.py:215-316): LN1 -> fused QKV GEMM -> q/k head-LN -> attention ->
    o_proj (+residual) -> LN2 -> FFN (bias, act) -> (+residual)."""

    def __init__(self, embedding_dim: int = 768, n_head: int = 8, activation_func: Callable = F.gelu,
                 multiplication_factor: int = 4, ff_dropout: float = 0.2, att_dropout: float = 0.2,
                 fast_att: bool = True, normalize_qv: bool = True, drop_p: float = 0.1):
        super().__init__()
        assert embedding_dim % n_head == 0, "Number of embedding_dim must be divisible by n_head"
        self.embedding_dim = embedding_dim
        self.n_head = n_head
        self.head_dim = embedding_dim // n_head
        self.att_dropout = att_dropout
        self.fast_att = fast_att
        self.q_norm = nn.LayerNorm(self.head_dim) if normalize_qv else nn.Identity()
        self.k_norm = nn.LayerNorm(self.head_dim) if normalize_qv else nn.Identity()
        self.drop_path1, self.drop_path2 = (SD(drop_p), SD(drop_p)) if drop_p > 1e-5 else (nn.Identity(), nn.Identity())
        self.q_proj = nn.Linear(embedding_dim, embedding_dim, bias=False)
        self.k_proj = nn.Linear(embedding_dim, embedding_dim, bias=False)
        self.v_proj = nn.Linear(embedding_dim, embedding_dim, bias=False)
        self.o_proj = nn.Linear(embedding_dim, embedding_dim, bias=False)
        self.ff_linear1 = nn.Linear(embedding_dim, multiplication_factor * embedding_dim, bias=True)
        self.ff_linear2 = nn.Linear(multiplication_factor * embedding_dim, embedding_dim, bias=True)
        self.norm1 = nn.LayerNorm(embedding_dim)
        self.norm2 = nn.LayerNorm(embedding_dim)
        self.activation = activation_func
        self.dropout = nn.Dropout(ff_dropout)

    def _prep(self, dt):
        qn = isinstance(self.q_norm, nn.LayerNorm)
        params = [self.q_proj.weight, self.k_proj.weight, self.v_proj.weight, self.o_proj.weight,
                  self.ff_linear1.weight, self.ff_linear1.bias, self.ff_linear2.weight, self.ff_linear2.bias,
                  self.norm1.weight, self.norm1.bias, self.norm2.weight, self.norm2.bias]
        if qn:
            params += [self.q_norm.weight, self.q_norm.bias, self.k_norm.weight, self.k_norm.bias]

        def build():
            # norm1 folded into the fused QKV projection, norm2 into ff_linear1 (sdp_gemm_ln)
            wqkv32 = torch.cat([f32(self.q_proj.weight), f32(self.k_proj.weight), f32(self.v_proj.weight)], 0)
            wqkv, sqkv, cqkv = _fold(wqkv32.contiguous(), self.norm1, None, dt)
            w1, s1, c1 = _fold(self.ff_linear1.weight, self.norm2, self.ff_linear1.bias, dt)
            if not _LN_FOLD:
                wqkv, sqkv, cqkv = as_dtype(wqkv32.contiguous(), dt), None, None
                w1, s1, c1 = as_dtype(self.ff_linear1.weight, dt), None, f32(self.ff_linear1.bias)
            d = dict(wqkv=wqkv, sqkv=sqkv, cqkv=cqkv, wo=as_dtype(self.o_proj.weight, dt),
                     n1g=f32(self.norm1.weight), n1b=f32(self.norm1.bias),
                     n2g=f32(self.norm2.weight), n2b=f32(self.norm2.bias),
                     w1=w1, s1=s1, c1=c1,
                     w2=as_dtype(self.ff_linear2.weight, dt), b2=f32(self.ff_linear2.bias),
                     n1e=self.norm1.eps, n2e=self.norm2.eps)
            if qn:
                d.update(qg=f32(self.q_norm.weight), qb=f32(self.q_norm.bias), kg=f32(self.k_norm.weight),
                         kb=f32(self.k_norm.bias), qe=self.q_norm.eps)
            return d
        return cached(self, "w", params, dt, build)

    def _mask_bias(self, mask: torch.Tensor, B: int, N: int):
        """Additive fp32 bias view [B', H', N, N] + (batch, head) strides."""
        if self.fast_att:                      # SDPA semantics (layers.py:291)
            if mask.dtype == torch.bool:
                add = torch.zeros(mask.shape, dtype=torch.float32, device=mask.device).masked_fill(~mask, float("-inf"))
            else:
                add = mask.float()
        else:                                  # masked_fill(mask == 0, -inf) (layers.py:294-295)
            add = torch.zeros(mask.shape, dtype=torch.float32, device=mask.device).masked_fill(mask == 0, float("-inf"))
        while add.dim() < 4:
            add = add.unsqueeze(0)
        add = add.expand(B, self.n_head, N, N)
        if not (add.stride(-1) == 1 and add.stride(-2) == N):
            add = add.contiguous()
        return add, add.stride(0), add.stride(1)

    def _run_tokens(self, tok: torch.Tensor, B: int, N: int, dt, mask: Optional[torch.Tensor] = None,
                    part: Optional[torch.Tensor] = None):
        """In place on the dense token buffer ``tok`` [B*N, C] (registers first).
        ``part``: its LN partial statistics (computed here when not given)."""
        C, Hn, hd = self.embedding_dim, self.n_head, self.head_dim
        T = B * N
        w = self._prep(dt)
        dev = tok.device
        if part is None:
            part = new_partials(T, C, dev)
            sp.row_partials(_dense(tok), T, C, part)
        # LN1 (:280) folded into the fused QKV projection (:282-284)
        qkv = torch.empty(T, 3 * C, dtype=dt, device=dev)
        if _LN_FOLD:
            st1 = _ln_stats(part, _dense(tok), T, C, w["n1e"])
            sp.gemm(_dense(tok), w["wqkv"], _dense(qkv), T, 3 * C, C, bias=w["cqkv"], ln=(st1, w["sqkv"]))
        else:
            h = torch.empty(T, C, dtype=dt, device=dev)
            sp.layernorm(_dense(tok), w["n1g"], w["n1b"], w["n1e"], _dense(h), T, C)
            sp.gemm(_dense(h), w["wqkv"], _dense(qkv), T, 3 * C, C)
        qkn = (w["qg"], w["qb"], w["kg"], w["kb"]) if "qg" in w else None                  # :286 (fused)
        att = torch.empty(T, C, dtype=dt, device=dev)
        if mask is not None:
            mb, sb, sh = self._mask_bias(mask, B, N)
            sp.attention(qkv, att, B, N, Hn, hd, mb, sb, sh, qk_norm=qkn, eps=w.get("qe", 1e-5))  # :289-298
        else:
            sp.attention(qkv, att, B, N, Hn, hd, qk_norm=qkn, eps=w.get("qe", 1e-5))
        sp.gemm(_dense(att), w["wo"], _dense(tok), T, C, C, resid=_dense(tok), part=part)  # :300-303
        # LN2 (:307) folded into ff_linear1 (:308)
        F_ = w["w1"].shape[0]
        f = torch.empty(T, F_, dtype=dt, device=dev)
        if _LN_FOLD:
            st2 = _ln_stats(part, _dense(tok), T, C, w["n2e"])
            sp.gemm(_dense(tok), w["w1"], _dense(f), T, F_, C, bias=w["c1"], act=act_code(self.activation),
                    ln=(st2, w["s1"]))
        else:
            h = torch.empty(T, C, dtype=dt, device=dev)
            sp.layernorm(_dense(tok), w["n2g"], w["n2b"], w["n2e"], _dense(h), T, C)
            sp.gemm(_dense(h), w["w1"], _dense(f), T, F_, C, bias=w["c1"], act=act_code(self.activation))
        sp.gemm(_dense(f), w["w2"], _dense(tok), T, C, F_, bias=w["b2"], resid=_dense(tok), part=part)  # :308-309

    def forward(self, x: torch.Tensor, register: torch.Tensor, mask: torch.Tensor = None):
        if self.training:
            return _train().train_encoder(self, x, register, mask)
        dt = compute_dtype(x, self)
        with torch.no_grad():
            tok, B, N, R, H, W = _to_tokens(x, register, dt)
            self._run_tokens(tok, B, N, dt, mask)
            return _from_tokens(tok, B, N, R, H, W, x.shape[1], dt)


def _to_tokens(x: torch.Tensor, register: torch.Tensor, dt):
    """NCHW x + registers [B,R,C] -> dense token buffer [B*(R+HW), C] (layers.py:271-275)."""
    B, C, H, W = x.shape
    R = register.shape[1]
    N = R + H * W
    tok = torch.empty(B * N, C, dtype=dt, device=x.device)
    sp.nchw_to_rows(x.to(dt).contiguous(), Rows(tok, C, H * W, N, R))
    if R:
        sp.copy_rows(register.to(dt).contiguous(), C, R * C, tok, C, N * C, B, R, C)
    return tok, B, N, R, H, W


def _from_tokens(tok: torch.Tensor, B, N, R, H, W, C, dt):
    """Split back into (x NCHW, registers [B,R,C]) (layers.py:311-314)."""
    x = torch.empty(B, C, H, W, dtype=dt, device=tok.device)
    sp.rows_to_nchw(Rows(tok, C, H * W, N, R), x)
    reg = torch.empty(B, R, C, dtype=dt, device=tok.device)
    if R:
        sp.copy_rows(tok, C, N * C, reg, C, R * C, B, R, C)
    return x, reg


class Block(nn.Module):
    """SdP-Net block: conv_block_num ConvMixers + an EncoderLayer, order set by
    conv_first (layers.py:337-386)."""

    def __init__(self, embedding_dim: int = 768, n_head: int = 8, conv_block_num: int = 2,
                 activation_func: Callable = nn.GELU(), multiplication_factor: int = 2, ff_dropout: float = 0.2,
                 att_dropout: float = 0.2, conv_kernel_size: int = 5, conv_activation: Callable = nn.GELU(),
                 conv_first=False, normalize_qv: bool = True, mixer_ffn_bias: bool = False,
                 mixer_deptwise_bias: bool = False, drop_p: float = 0.1, fast_att: bool = True):
        super().__init__()
        self.t_block = EncoderLayer(embedding_dim=embedding_dim, n_head=n_head, activation_func=activation_func,
                                    multiplication_factor=multiplication_factor, ff_dropout=ff_dropout,
                                    att_dropout=att_dropout, normalize_qv=normalize_qv, drop_p=drop_p,
                                    fast_att=fast_att)
        self.conv_blocks = nn.Sequential(*[ConvMixer(embedding_dim=embedding_dim, kernel_size=conv_kernel_size,
                                                     activation=conv_activation, drop_p=drop_p,
                                                     mixer_deptwise_bias=mixer_deptwise_bias,
                                                     mixer_ffn_bias=mixer_ffn_bias)
                                           for _ in range(conv_block_num)])
        self.conv_first = conv_first

    def _run_tokens(self, tok: torch.Tensor, B: int, R: int, H: int, W: int, dt, mask=None,
                    part: Optional[torch.Tensor] = None):
        N = R + H * W
        C = tok.shape[-1]
        img = Rows(tok, C, H * W, N, R)
        if part is None:
            part = new_partials(B * N, C, tok.device)
            sp.row_partials(_dense(tok), B * N, C, part)
        if not self.conv_first:
            self.t_block._run_tokens(tok, B, N, dt, mask, part=part)
            for m in self.conv_blocks:
                m._run_tokens(img, B, H, W, dt, part=part)
            return
        for m in self.conv_blocks:
            m._run_tokens(img, B, H, W, dt, part=part)
        self.t_block._run_tokens(tok, B, N, dt, mask, part=part)

    def forward(self, x: torch.Tensor, register: torch.Tensor, mask: torch.Tensor = None):
        if hooked(self):  # reference composition (layers.py:381-386) so hooked children fire
            if not self.conv_first:
                x, register = self.t_block(x, register, mask)
                x = self.conv_blocks(x)
                return x, register
            x = self.conv_blocks(x)
            return self.t_block(x, register, mask)
        if self.training:
            return _train().train_block(self, x, register, mask)
        dt = compute_dtype(x, self)
        with torch.no_grad():
            tok, B, N, R, H, W = _to_tokens(x, register, dt)
            self._run_tokens(tok, B, R, H, W, dt, mask)
            return _from_tokens(tok, B, N, R, H, W, x.shape[1], dt)


class FinalBlock(nn.Module):
    """A lone EncoderLayer (layers.py:400-426)."""

    def __init__(self, embedding_dim: int = 768, n_head: int = 8, activation_func: Callable = F.gelu,
                 multiplication_factor: int = 2, ff_dropout: float = 0.2, att_dropout: float = 0.2,
                 normalize_qv: bool = True, drop_p: float = 0.0):
        super().__init__()
        self.t_block = EncoderLayer(embedding_dim=embedding_dim, n_head=n_head, activation_func=activation_func,
                                    multiplication_factor=multiplication_factor, ff_dropout=ff_dropout,
                                    att_dropout=att_dropout, normalize_qv=normalize_qv, drop_p=drop_p)

    def _run_tokens(self, tok, B, R, H, W, dt, mask=None, part: Optional[torch.Tensor] = None):
        self.t_block._run_tokens(tok, B, R + H * W, dt, mask, part=part)

    def forward(self, x: torch.Tensor, register: torch.Tensor, mask: torch.Tensor = None):
        return self.t_block(x, register, mask)


class ClassificationHead(nn.Module):
    """Head (layers.py:429-465).  from_register: LN(mean_R(registers)) -> Linear
    [-> Tanh -> Dropout -> Linear]; else AdaptiveAvgPool over x -> Linear."""

    def __init__(self, embedding_dim: int = 768, output_classes: int = 1000, dropout: float = 0.2,
                 from_register: bool = True, simple_output: bool = False, bias: bool = False):
        super().__init__()
        self.from_register = from_register
        if from_register:
            if simple_output:
                self.output_head = nn.Sequential(*[nn.LayerNorm(embedding_dim),
                                                   nn.Linear(embedding_dim, output_classes, bias=bias)])
            else:
                self.output_head = nn.Sequential(*[nn.LayerNorm(embedding_dim),
                                                   nn.Linear(embedding_dim, output_classes, bias=bias),
                                                   nn.Tanh(),
                                                   nn.Dropout(dropout),
                                                   nn.Linear(output_classes, output_classes, bias=bias)])
        else:
            self.output_head = nn.Sequential(*[nn.AdaptiveAvgPool2d((1, 1)), nn.Flatten(),
                                               nn.Linear(embedding_dim, output_classes, bias=bias)])

    def _prep(self, dt):
        lins = [m for m in self.output_head if isinstance(m, nn.Linear)]
        lns = [m for m in self.output_head if isinstance(m, nn.LayerNorm)]
        params = []
        for m in lins + lns:
            params += [m.weight, m.bias]

        def build():
            lin = [(as_dtype(m.weight, dt), f32(m.bias)) for m in lins]
            pad = -lin[0][0].shape[0] % 64
            if len(lin) == 2 and dt == torch.bfloat16 and pad:
                # The bf16 MFMA GEMM needs K % 64 == 0. Zero-pad the hidden width (1000 -> 1024):
                # the extra hidden units have zero weights and bias, so tanh(0) = 0, and they
                # meet zero K columns of the second weight. The logits are unchanged and both
                # GEMMs take the fast path instead of gemm_generic.
                (w1, b1), (w2, b2) = lin
                w1 = F.pad(w1, (0, 0, 0, pad))
                b1 = None if b1 is None else F.pad(b1, (0, pad))
                lin = [(w1, b1), (F.pad(w2, (0, pad)).contiguous(), b2)]
            d = dict(lin=lin)
            if lns:
                d["ln"] = (f32(lns[0].weight), f32(lns[0].bias), lns[0].eps)
            return d
        return cached(self, "w", params, dt, build)

    def _run(self, src: Rows, B: int, rows: int, C: int, dt, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """src: B groups of `rows` logical rows to average (registers or pixels).
        Logits go to ``out`` [B, classes] when given (written in place)."""
        w = self._prep(dt)
        dev = src.t.device
        h = torch.empty(B, C, dtype=dt, device=dev)
        sp.group_mean(src, h, B, rows, C)
        if self.from_register:
            g, b, eps = w["ln"]
            sp.layernorm(_dense(h), g, b, eps, _dense(h), B, C)
        (w1, b1) = w["lin"][0]
        n1 = w1.shape[0]
        two = len(w["lin"]) == 2
        y = out if (out is not None and not two) else torch.empty(B, n1, dtype=dt, device=dev)
        sp.gemm(_dense(h), w1, _dense(y), B, n1, C, bias=b1, act=sp.ACT_CODES["tanh"] if two else 0)
        if not two:
            return y
        (w2, b2) = w["lin"][1]
        res = out if out is not None else torch.empty(B, w2.shape[0], dtype=dt, device=dev)
        sp.gemm(_dense(y), w2, _dense(res), B, w2.shape[0], n1, bias=b2)
        return res

    def forward(self, x: torch.Tensor, registers: torch.Tensor) -> torch.Tensor:
        if self.training:
            return _train().train_head(self, x, registers)
        dt = compute_dtype(x if not self.from_register else registers, self)
        with torch.no_grad():
            if self.from_register:
                B, R, C = registers.shape
                r = registers.to(dt).contiguous()
                return self._run(Rows(r, C), B, R, C, dt)
            B, C, H, W = x.shape
            rows = torch.empty(B * H * W, C, dtype=dt, device=x.device)
            sp.nchw_to_rows(x.to(dt).contiguous(), _dense(rows))
            return self._run(_dense(rows), B, H * W, C, dt)
