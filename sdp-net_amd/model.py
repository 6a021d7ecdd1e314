"""Drop-in ``model`` module: ``MainModel`` of y-akbal/SdP-Net (model.py:27-149)
with the same 25 constructor kwargs and defaults, activation registry,
module tree / state_dict keys, weight init and forward signature.

The forward is the fused MI355X path: one persistent token buffer
[B, R + (Hi/p)*(Wi/p), C] (registers first) in HBM; every op is a gfx950 HIP
kernel from libsdpnet_hip.so:

  patchify -> patch GEMM (+pos-emb, +embedding act, written into the image rows)
  -> register rows -> N x Block [2 x ConvMixer (LN -> DW kxk -> GEMM(+act,+res)
  -> LN -> GEMM(+act) -> GEMM(+res)) + Encoder (LN -> QKV GEMM -> q/k LN ->
  attention -> O GEMM(+res) -> LN -> FF1(+bias,act) -> FF2(+bias,+res))]
  -> FinalBlock -> head (mean / LN / GEMM(+tanh) / GEMM).

fp32 inputs run the fp32 path (exact f32 MFMA); bf16 inputs, bf16 params or a
CUDA bf16 autocast region run the bf16 path (bf16 storage, fp32 accumulate).
"""
from __future__ import annotations

import os
from typing import Callable

import torch
from torch import nn as nn
from torch.nn import functional as F
from numpy import arccos, cos

import sdpnet_hip as sp
import sdpnet_ops
from layers import ConvMixer, EmbeddingLayer, ConvPatcher, Block, FinalBlock, ClassificationHead, ConvEmbedding  # noqa: F401
from utility_layers import SdPModel, StochasticDepth  # noqa: F401
from layers import new_partials  # token-buffer plumbing of the fused path
from sdpnet_engine import act_code, as_dtype, cached, compute_dtype, hooked as _hooked
from training_utilities import KeLu

# torch.compile of a training model: "layer" (default) = one custom op per sub-layer (DDP's
# bucket all-reduce overlaps the compiled backward), "model" = one op pair for the whole model
_COMPILE_TRAIN_OPS = os.environ.get("SDPNET_COMPILE_TRAIN_OPS", "layer")
# bf16 eval forward with autocast's fp32 residual stream (training_tools.py:85): model.eval_fp32_stream
# = True, or this default for every model
_EVAL_FP32_STREAM = os.environ.get("SDPNET_EVAL_FP32_STREAM", "0") != "0"

torch.set_float32_matmul_precision('high')  # model.py:9 (import side effect kept)

# model.py:13-24
activations = {
    "relu": nn.ReLU(),
    "gelu": nn.GELU(),
    "fast_gelu": nn.GELU("fast"),
    "tanh": nn.Tanh(),
    "sigmoid": nn.Sigmoid(),
    "leaky_relu": nn.LeakyReLU(),
    "selu": nn.SELU(),
    "none": nn.Identity(),
    "kelu": KeLu,
}

Rows = sp.Rows


class MainModel(SdPModel):
    def __init__(self,
                 embedding_dim: int = 128,
                 num_blocks: int = 10,
                 n_head: int = 4,
                 activation: Callable = "gelu",
                 conv_kernel_size: int = 5,
                 patch_size: int = 16,
                 ffn_dropout: float = 0.2,
                 attn_dropout: float = 0.2,
                 output_classes: int = 1000,
                 conv_block_num: int = 2,
                 ff_multiplication_factor: int = 4,
                 max_image_size: list = [14, 14],
                 max_num_registers: int = 5,
                 embedding_activation: Callable = "none",
                 conv_first: bool = True,
                 head_output_from_register: bool = False,
                 simple_mlp_output: bool = False,
                 output_head_bias: bool = False,
                 normalize_qv: bool = True,
                 stochastic_depth_p: list = [0.0, 0.0],
                 mixer_deptwise_bias: bool = False,
                 mixer_ffn_bias: bool = False,
                 fast_att: bool = True,
                 conv_embedding: bool = False,
                 conv_embedding_kernel_size: int = 5,
                 ):
        super().__init__()
        activation = activations[activation.lower()] if isinstance(activation, str) else activation
        embedding_activation = (activations[embedding_activation.lower()]
                                if isinstance(embedding_activation, str) else embedding_activation)
        self.conv_init = ConvPatcher(embedding_dim=embedding_dim, patch_size=patch_size)
        if not conv_embedding:
            self.embedding_layer = EmbeddingLayer(embedding_dim=embedding_dim, max_num_registers=max_num_registers,
                                                  max_image_size=max_image_size, activation=embedding_activation)
        else:
            self.embedding_layer = ConvEmbedding(embedding_dim=embedding_dim, max_num_registers=max_num_registers,
                                                 max_image_size=max_image_size, kernel_size=conv_embedding_kernel_size,
                                                 activation=embedding_activation)
        # cosine schedule of the stochastic-depth p (model.py:82)
        ST_p = lambda i: cos(arccos(stochastic_depth_p[0]) * (1 - i / num_blocks)  # noqa: E731
                             + arccos(stochastic_depth_p[1]) * (i / num_blocks))
        self.blocks = nn.ModuleList([
            Block(embedding_dim=embedding_dim, n_head=n_head, activation_func=activation, ff_dropout=ffn_dropout,
                  att_dropout=attn_dropout, multiplication_factor=ff_multiplication_factor,
                  conv_kernel_size=conv_kernel_size, conv_activation=activation, conv_first=conv_first,
                  conv_block_num=conv_block_num, normalize_qv=normalize_qv, drop_p=ST_p(i),
                  mixer_deptwise_bias=mixer_deptwise_bias, mixer_ffn_bias=mixer_ffn_bias, fast_att=fast_att)
            for i in range(num_blocks)])
        self.final_block = FinalBlock(embedding_dim=embedding_dim, n_head=n_head, activation_func=activation,
                                      multiplication_factor=ff_multiplication_factor, ff_dropout=ffn_dropout,
                                      att_dropout=attn_dropout, normalize_qv=normalize_qv, drop_p=0.0)
        self.output_head = ClassificationHead(embedding_dim, output_classes, ffn_dropout,
                                              from_register=head_output_from_register,
                                              simple_output=simple_mlp_output, bias=output_head_bias)
        self.__init_weights__()
        self._sdp_handle = sdpnet_ops.register(self)

    def __setstate__(self, state):
        # deep copies / unpickled models get their own custom-op handle
        super().__setstate__(state)
        self._sdp_handle = sdpnet_ops.register(self)

    def __init_weights__(self):
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.trunc_normal_(m.weight, std=0.01)
            elif isinstance(m, nn.Conv2d):
                nn.init.trunc_normal_(m.weight, std=0.01)

    # ------------------------------------------------------------------
    def _pos_rows(self, Hp: int, Wp: int, dt) -> torch.Tensor:
        emb = self.embedding_layer
        pos = emb._pos_table(Hp, Wp)
        if dt == torch.float32:
            return pos
        return cached(emb, f"pos{Hp}x{Wp}_{dt}", [pos], dt, lambda: as_dtype(pos, dt))

    def _prepare(self, dt, Hp: int, Wp: int):
        """Build every prepared-weight cache on the current stream (before any fork)."""
        self.conv_init._weight(dt)
        self._pos_rows(Hp, Wp, dt)
        for blk in self.blocks:
            blk.t_block._prep(dt)
            for mx in blk.conv_blocks:
                mx._prep(dt)
                mx.layer_norm_1._params()
                mx.layer_norm_2._params()
        self.final_block.t_block._prep(dt)
        self.output_head._prep(dt)

    def _num_streams(self, B: int) -> int:
        n = getattr(self, "num_streams", None)
        if n is None:
            env = os.environ.get("SDPNET_STREAMS")
            n = int(env) if env else (2 if B >= 64 else 1)
        return max(1, min(int(n), B))

    def forward(self, x: torch.Tensor, num_registers: int = 3, return_raw_outputs: bool = False):
        if self.training:
            # training_tools.py:77-103: the train-mode forward with dropout / drop path, whose
            # backward runs on the HIP kernels too (sdpnet_train.py)
            if torch.compiler.is_compiling():
                # torch.compile of a training model (cifar100_test.py:93, training_tools.py:39):
                # one opaque op per sub-layer, each with an op as its autograd formula
                # (sdpnet_ops.train_layer), or the whole model as one op pair
                # (SDPNET_COMPILE_TRAIN_OPS=model: sdpnet_ops.train_forward / train_backward)
                # (raw outputs and an image that requires grad take the per-layer ops: the head op with
                # raw outputs, layer 0's backward with the image gradient)
                code = sdpnet_ops.DTYPE_CODES[compute_dtype(x, self)]
                if _COMPILE_TRAIN_OPS == "model" and not return_raw_outputs and not x.requires_grad:
                    params = [p for p in self.parameters()]
                    logits, _ = torch.ops.sdpnet.train_forward(x, params, self._sdp_handle, num_registers, code)
                    return logits
                import sdpnet_train
                return sdpnet_train.compiled_train_forward(self, x, num_registers, code, return_raw_outputs)
            import sdpnet_train
            return sdpnet_train.train_forward(self, x, num_registers, return_raw_outputs)
        if torch.compiler.is_compiling():
            # torch.compile (model_test.py:64, cifar100_test.py:93 fullgraph=True): the whole
            # fused forward is one opaque custom op with a shape-only fake (sdpnet_ops.py)
            code = sdpnet_ops.DTYPE_CODES[compute_dtype(x, self)]
            if return_raw_outputs:
                return torch.ops.sdpnet.main_forward_raw(x, self._sdp_handle, num_registers, code)
            return torch.ops.sdpnet.main_forward(x, self._sdp_handle, num_registers, code)
        if _hooked(self):
            return self._forward_modules(x, num_registers, return_raw_outputs)
        if self._fp32_stream_eval(x):
            import sdpnet_train
            return sdpnet_train.eval_forward(self, x, num_registers, return_raw_outputs)
        return self._fused_forward(x, num_registers, compute_dtype(x, self), return_raw_outputs)

    def _fp32_stream_eval(self, x: torch.Tensor) -> bool:
        """bf16 eval forward along the training forward's kernels with the residual stream (the token
        rows between sub-layers) in fp32, as torch.autocast keeps it (training_tools.py:85; residual adds
        layers.py:102-103, :303, :309), bf16 GEMM operands, no dropout / drop path
        (sdpnet_train.eval_forward).  Opt-in (model.eval_fp32_stream = True or
        SDPNET_EVAL_FP32_STREAM=1): the fused forward keeps the stream in bf16, ~2.3x the reference's own
        autocast logit error at M and faster."""
        on = getattr(self, "eval_fp32_stream", None)
        if on is None:
            on = _EVAL_FP32_STREAM
        return bool(on) and x.is_cuda and compute_dtype(x, self) == torch.bfloat16

    def _fused_forward(self, x: torch.Tensor, num_registers: int, dt, return_raw_outputs: bool):
        with torch.no_grad():
            B, _, Hi, Wi = x.shape
            p = self.conv_init.patch_size
            Hp, Wp = Hi // p, Wi // p
            C = self.conv_init.conv.out_channels
            ncls = self.output_head._prep(dt)["lin"][-1][0].shape[0]
            self._prepare(dt, Hp, Wp)
            x = x.contiguous()
            logits = torch.empty(B, ncls, dtype=dt, device=x.device)
            ns = 1 if return_raw_outputs else self._num_streams(B)
            if ns == 1:
                raw = self._forward_chunk(x, logits, num_registers, dt, Hp, Wp, C, return_raw_outputs)
                return logits if not return_raw_outputs else (logits, *raw)
            # Independent sub-batches on concurrent HIP streams: one chunk's tail waves and
            # memory-bound kernels overlap the other's GEMMs (no data dependence between images).
            main = torch.cuda.current_stream(x.device)
            streams = self.__dict__.setdefault("_sdp_streams", {})
            if (x.device, ns) not in streams:
                streams[(x.device, ns)] = [torch.cuda.Stream(device=x.device) for _ in range(ns)]
            streams = streams[(x.device, ns)]
            step = (B + ns - 1) // ns
            for i, s in enumerate(streams):
                lo, hi = i * step, min(B, (i + 1) * step)
                if lo >= hi:
                    continue
                s.wait_stream(main)
                with torch.cuda.stream(s):
                    self._forward_chunk(x[lo:hi], logits[lo:hi], num_registers, dt, Hp, Wp, C, False)
            for s in streams:
                main.wait_stream(s)
            return logits

    def _forward_chunk(self, x, logits, num_registers, dt, Hp, Wp, C, return_raw_outputs):
        """Fused forward of one (sub-)batch on the current stream; logits written in place."""
        B = x.shape[0]
        P = Hp * Wp
        emb = self.embedding_layer
        table, R = emb._register_rows(num_registers)
        N = R + P
        tok = torch.empty(B * N, C, dtype=dt, device=x.device)
        img = Rows(tok, C, P, N, R)
        # patch GEMM + positional table (+ embedding activation) into the image rows
        # (layers.py:40-42, :157-168 / :205)
        part = new_partials(B * N, C, x.device)  # LN statistics by parts of every token row
        self.conv_init._run(x, dt, img, resid=Rows(self._pos_rows(Hp, Wp, dt), C, P, 0, 0),
                            act=act_code(emb.activation), part=part)
        if R:
            sp.copy_rows(table.contiguous(), C, 0, tok, C, N * C, B, R, C)
            sp.row_partials(Rows(tok, C, R, N, 0), B * R, C, part)
        for block in self.blocks:                                     # model.py:139-140
            block._run_tokens(tok, B, R, Hp, Wp, dt, part=part)
        self.final_block._run_tokens(tok, B, R, Hp, Wp, dt, part=part)  # model.py:143
        head = self.output_head                                       # model.py:146
        if head.from_register:
            head._run(Rows(tok, C, R, N, 0), B, R, C, dt, out=logits)
        else:
            head._run(img, B, P, C, dt, out=logits)
        if not return_raw_outputs:
            return None
        xo = torch.empty(B, C, Hp, Wp, dtype=dt, device=x.device)
        sp.rows_to_nchw(img, xo)
        regs = torch.empty(B, R, C, dtype=dt, device=x.device)
        if R:
            sp.copy_rows(tok, C, N * C, regs, C, R * C, B, R, C)
        return xo, regs

    def _forward_modules(self, x, num_registers, return_raw_outputs):
        """Module-by-module composition (model.py:129-149) used while forward hooks
        are attached (layer_test), so every submodule's __call__ fires."""
        x = self.conv_init(x)
        x_raw_output, registers = self.embedding_layer(x, num_registers)
        for block in self.blocks:
            x_raw_output, registers = block(x_raw_output, registers)
        x_raw_output, registers = self.final_block(x_raw_output, registers)
        x_classification_head = self.output_head(x_raw_output, registers)
        if not return_raw_outputs:
            return x_classification_head
        return x_classification_head, x_raw_output, registers


if __name__ == "__main__":
    print("Ok boomer!!!")
