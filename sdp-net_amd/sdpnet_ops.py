"""torch.library registration of the fused MainModel forward.

The reference's harnesses wrap the model in ``torch.compile`` -- ``model_test.py:64``,
``training_tools.py:39`` (``dynamic=True``) and ``cifar100_test.py:93``
(``fullgraph=True``).  The fused forward is a chain of ctypes launches into
libsdpnet_hip.so that Dynamo cannot trace, so under compilation ``MainModel.forward``
emits ONE opaque custom op per call instead:

    sdpnet::main_forward(Tensor x, int handle, int num_registers, int dtype_code) -> Tensor
    sdpnet::main_forward_raw(...) -> (Tensor logits, Tensor x_nchw, Tensor registers)

``handle`` names the live MainModel in a process-local registry (weak references;
a deep copy or unpickled copy registers itself anew, ``MainModel.__setstate__``).
The fake (meta) implementations give the output shapes from the module structure
alone, so ``fullgraph=True`` and ``dynamic=True`` trace with 0 graph breaks.  The
real implementation is registered for the CUDA (ROCm) device type only: a CPU
tensor reaching it raises instead of silently running some other path.
"""
from __future__ import annotations

import itertools
import weakref
from typing import Tuple

import torch
from torch import Tensor

from sdpnet_engine import num_reg_rows
from typing import List, Optional

_MODELS: "dict[int, weakref.ref]" = {}
_NEXT = itertools.count(1)

DTYPE_CODES = {torch.float32: 0, torch.bfloat16: 1}
_DTYPES = {v: k for k, v in DTYPE_CODES.items()}


def register(model) -> int:
    """Give ``model`` a fresh handle (called from MainModel.__init__ / __setstate__)."""
    h = next(_NEXT)
    _MODELS[h] = weakref.ref(model, lambda _r, h=h: _MODELS.pop(h, None))
    return h


def lookup(handle: int):
    ref = _MODELS.get(int(handle))
    model = ref() if ref is not None else None
    if model is None:
        raise RuntimeError(f"sdpnet: model handle {handle} is not live (the MainModel was freed)")
    return model


def _register_rows(model, num_registers: int) -> int:
    emb = model.embedding_layer
    n = emb.register.shape[0] if hasattr(emb, "register") else emb.max_num_registers
    return num_reg_rows(n, num_registers)


def _shapes(model, x: Tensor, num_registers: int):
    B, _, Hi, Wi = x.shape
    p = model.conv_init.patch_size
    C = model.conv_init.conv.out_channels
    lins = [m for m in model.output_head.output_head if isinstance(m, torch.nn.Linear)]
    ncls = lins[-1].out_features
    return B, C, Hi // p, Wi // p, ncls, _register_rows(model, num_registers)


@torch.library.custom_op("sdpnet::main_forward", mutates_args=(), device_types="cuda")
def main_forward(x: Tensor, handle: int, num_registers: int, dtype_code: int) -> Tensor:
    return lookup(handle)._fused_forward(x, num_registers, _DTYPES[dtype_code], False)


@main_forward.register_fake
def _main_forward_fake(x, handle, num_registers, dtype_code):
    B, C, Hp, Wp, ncls, R = _shapes(lookup(handle), x, num_registers)
    return x.new_empty((B, ncls), dtype=_DTYPES[dtype_code])


@torch.library.custom_op("sdpnet::main_forward_raw", mutates_args=(), device_types="cuda")
def main_forward_raw(x: Tensor, handle: int, num_registers: int, dtype_code: int) -> Tuple[Tensor, Tensor, Tensor]:
    logits, xo, regs = lookup(handle)._fused_forward(x, num_registers, _DTYPES[dtype_code], True)
    return logits, xo, regs


@main_forward_raw.register_fake
def _main_forward_raw_fake(x, handle, num_registers, dtype_code):
    B, C, Hp, Wp, ncls, R = _shapes(lookup(handle), x, num_registers)
    dt = _DTYPES[dtype_code]
    return (x.new_empty((B, ncls), dtype=dt), x.new_empty((B, C, Hp, Wp), dtype=dt),
            x.new_empty((B, R, C), dtype=dt))


# ---------------------------------------------------------------------------
# Training mode under torch.compile (cifar100_test.py:93 fullgraph=True, dynamic=True;
# training_tools.py:38-39): the whole train-mode forward is ONE opaque op whose autograd
# formula is a second opaque op, so Dynamo traces model(x) -> loss.backward() with 0 graph
# breaks and AOTAutograd never looks inside.
#
#   sdpnet::train_forward(x, params, handle, num_registers, dtype_code) -> (logits, key)
#   sdpnet::train_backward(grad_logits, key, params, handle) -> grads (one per param)
#
# The forward runs sdpnet_train.tape_forward (the eager path's own sub-layer Functions,
# called directly) and parks the tape in _TAPES under ``key``, a 1-element tensor that is
# also a saved tensor of the autograd node: backward finds the tape by key.data_ptr() (no
# host sync) and frees it; a tape whose key dies without a backward is dropped with it.
# ---------------------------------------------------------------------------
_TAPES: "dict[int, list]" = {}


def _drop_tape(k: int):
    _TAPES.pop(k, None)


@torch.library.custom_op("sdpnet::train_forward", mutates_args=(), device_types="cuda")
def train_forward(x: Tensor, params: List[Tensor], handle: int, num_registers: int,
                  dtype_code: int) -> Tuple[Tensor, Tensor]:
    import sdpnet_train
    model = lookup(handle)
    logits, tape = sdpnet_train.tape_forward(model, x, num_registers, _DTYPES[dtype_code])
    key = torch.empty(1, dtype=torch.int64, device=x.device)
    _TAPES[key.data_ptr()] = tape
    weakref.finalize(key, _drop_tape, key.data_ptr())
    return logits, key


@train_forward.register_fake
def _train_forward_fake(x, params, handle, num_registers, dtype_code):
    B, C, Hp, Wp, ncls, R = _shapes(lookup(handle), x, num_registers)
    return x.new_empty((B, ncls), dtype=_DTYPES[dtype_code]), x.new_empty((1,), dtype=torch.int64)


@torch.library.custom_op("sdpnet::train_backward", mutates_args=(), device_types="cuda")
def train_backward(grad_logits: Tensor, key: Tensor, params: List[Tensor], handle: int) -> List[Tensor]:
    import sdpnet_train
    tape = _TAPES.pop(key.data_ptr(), None)
    if tape is None:
        raise RuntimeError("sdpnet: no saved training forward for this backward (backward run twice?)")
    return sdpnet_train.tape_backward(tape, grad_logits.contiguous(), params)


@train_backward.register_fake
def _train_backward_fake(grad_logits, key, params, handle):
    return [torch.empty_like(p) for p in params]


def _train_setup_context(ctx, inputs, output):
    x, params, handle, num_registers, dtype_code = inputs
    ctx.save_for_backward(output[1], *params)
    ctx.handle = handle
    ctx.nparams = len(params)


def _train_backward_formula(ctx, grad_logits, grad_key):
    key, *params = ctx.saved_tensors
    grads = torch.ops.sdpnet.train_backward(grad_logits, key, params, ctx.handle)
    return None, list(grads), None, None, None


train_forward.register_autograd(_train_backward_formula, setup_context=_train_setup_context)


# ---------------------------------------------------------------------------
# Training mode under torch.compile, per sub-layer (the default; SDPNET_COMPILE_TRAIN_OPS=model
# selects the single op pair above): one op per patch-embedding / ConvMixer / EncoderLayer /
# head (sdpnet_train.train_layers order), each with an autograd formula that is a second op:
#
#   sdpnet::train_layer(t, params, handle, layer, num_registers, dtype_code, batch, need_dx) -> (out, key)
#   sdpnet::train_layer_backward(grad_out, key, params, handle, layer, in_shape, in_dtype) -> (grad_in, grads)
#
# (need_dx: layer 0's image requires grad, its backward op then returns the image gradient), so the
# compiled backward runs layer by layer and DDP (training_tools.py:36-39 compiles the
# DDP-wrapped model) all-reduces a bucket while earlier layers' backward ops still run.  The
# layer's ctx is parked under key.data_ptr() as for the whole-model pair.
# ---------------------------------------------------------------------------
@torch.library.custom_op("sdpnet::train_layer", mutates_args=(), device_types="cuda")
def train_layer(t: Tensor, params: List[Tensor], handle: int, layer: int, num_registers: int, dtype_code: int,
                batch: int, need_dx: int) -> Tuple[Tensor, Tensor]:
    import sdpnet_train
    out, rec = sdpnet_train.layer_forward(lookup(handle), layer, t, num_registers, _DTYPES[dtype_code],
                                          need_dx=bool(need_dx))
    key = torch.empty(1, dtype=torch.int64, device=t.device)
    _TAPES[key.data_ptr()] = rec
    weakref.finalize(key, _drop_tape, key.data_ptr())
    return out, key


@train_layer.register_fake
def _train_layer_fake(t, params, handle, layer, num_registers, dtype_code, batch, need_dx):
    import sdpnet_train
    model = lookup(handle)
    kind, _ = sdpnet_train.train_layers(model)[layer]
    key = t.new_empty((1,), dtype=torch.int64)
    dt = _DTYPES[dtype_code]
    if kind == "embed":
        B, C, Hp, Wp, ncls, R = _shapes(model, t, num_registers)
        return t.new_empty((B * (R + Hp * Wp), C), dtype=sdpnet_train.stream_dtype(dt, C)), key
    if kind == "head":
        lins = [m for m in model.output_head.output_head if isinstance(m, torch.nn.Linear)]
        return t.new_empty((batch, lins[-1].out_features), dtype=dt), key
    return torch.empty_like(t), key


@torch.library.custom_op("sdpnet::train_layer_backward", mutates_args=(), device_types="cuda")
def train_layer_backward(grad_out: Tensor, key: Tensor, params: List[Tensor], handle: int, layer: int,
                         in_shape: List[int], in_dtype: int) -> Tuple[Tensor, List[Tensor]]:
    import sdpnet_train
    rec = _TAPES.pop(key.data_ptr(), None)
    if rec is None:
        raise RuntimeError("sdpnet: no saved training forward for this layer's backward (backward run twice?)")
    gin, grads = sdpnet_train.layer_backward(rec, grad_out)
    if gin is None:  # layer 0 with an image that needs no gradient
        gin = grad_out.new_empty((0,))
    return gin, grads


# dtypes a layer input (and so its gradient) may have: the token rows are fp32 / bf16, an image that
# requires grad may also be fp16 / fp64 (patchify converts it to the compute dtype)
_GRAD_DTYPES = [torch.float32, torch.bfloat16, torch.float16, torch.float64]


@train_layer_backward.register_fake
def _train_layer_backward_fake(grad_out, key, params, handle, layer, in_shape, in_dtype):
    # (in_shape, in_dtype): the layer's forward input, i.e. its gradient's shape / dtype; the input
    # itself is not kept alive for the backward (eager frees it once the layer's ctx is done with it).
    # Layer 0 records an empty shape when the image needs no gradient.
    gin = grad_out.new_empty(in_shape, dtype=_GRAD_DTYPES[in_dtype]) if in_shape else grad_out.new_empty((0,))
    return gin, [torch.empty_like(p) for p in params]


def _layer_setup_context(ctx, inputs, output):
    t, params, handle, layer, num_registers, dtype_code, batch, need_dx = inputs
    ctx.save_for_backward(output[1], *params)
    ctx.handle = handle
    ctx.layer = layer
    ctx.want_gin = layer != 0 or bool(need_dx)
    ctx.in_shape = list(t.shape) if ctx.want_gin else []
    ctx.in_dtype = _GRAD_DTYPES.index(t.dtype) if ctx.want_gin else 0


def _layer_backward_formula(ctx, grad_out, grad_key):
    key, *params = ctx.saved_tensors
    gin, grads = torch.ops.sdpnet.train_layer_backward(grad_out, key, params, ctx.handle, ctx.layer, ctx.in_shape,
                                                       ctx.in_dtype)
    return (gin if ctx.want_gin else None), list(grads), None, None, None, None, None, None


train_layer.register_autograd(_layer_backward_formula, setup_context=_layer_setup_context)


# The head layer with the raw outputs (return_raw_outputs=True in train mode, model.py:145-149):
#   sdpnet::train_head_raw(t, params, handle, layer, num_registers, dtype_code, batch, hp, wp)
#       -> (logits, x_raw_output [B, C, hp, wp], registers [B, R, C], key)
#   sdpnet::train_head_raw_backward(grad_logits, grad_x_raw?, grad_registers?, key, params, handle,
#       in_shape, in_dtype) -> (grad_t, grads)
# The raw outputs are copies of the final token rows (_RawOutFn's kernels); their gradients are added
# to the head's token-row gradient by a HIP pass inside the backward op.
@torch.library.custom_op("sdpnet::train_head_raw", mutates_args=(), device_types="cuda")
def train_head_raw(t: Tensor, params: List[Tensor], handle: int, layer: int, num_registers: int, dtype_code: int,
                   batch: int, hp: int, wp: int) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    import sdpnet_train
    model = lookup(handle)
    C = model.conv_init.conv.out_channels
    geo = (batch, _register_rows(model, num_registers), hp, wp, C)
    xo, regs = sdpnet_train.raw_outputs(t, geo)
    logits, rec = sdpnet_train.layer_forward(model, layer, t, num_registers, _DTYPES[dtype_code])
    key = torch.empty(1, dtype=torch.int64, device=t.device)
    _TAPES[key.data_ptr()] = (rec, geo)
    weakref.finalize(key, _drop_tape, key.data_ptr())
    return logits, xo, regs, key


@train_head_raw.register_fake
def _train_head_raw_fake(t, params, handle, layer, num_registers, dtype_code, batch, hp, wp):
    model = lookup(handle)
    lins = [m for m in model.output_head.output_head if isinstance(m, torch.nn.Linear)]
    C = model.conv_init.conv.out_channels
    R = _register_rows(model, num_registers)
    return (t.new_empty((batch, lins[-1].out_features), dtype=_DTYPES[dtype_code]),
            t.new_empty((batch, C, hp, wp)), t.new_empty((batch, R, C)), t.new_empty((1,), dtype=torch.int64))


@torch.library.custom_op("sdpnet::train_head_raw_backward", mutates_args=(), device_types="cuda")
def train_head_raw_backward(grad_logits: Tensor, grad_xo: Optional[Tensor], grad_regs: Optional[Tensor], key: Tensor,
                            params: List[Tensor], handle: int, in_shape: List[int],
                            in_dtype: int) -> Tuple[Tensor, List[Tensor]]:
    import sdpnet_train
    tape = _TAPES.pop(key.data_ptr(), None)
    if tape is None:
        raise RuntimeError("sdpnet: no saved training forward for the head's backward (backward run twice?)")
    rec, geo = tape
    gin, grads = sdpnet_train.layer_backward(rec, grad_logits)
    return sdpnet_train.add_raw_output_grads(gin, grad_xo, grad_regs, geo), grads


@train_head_raw_backward.register_fake
def _train_head_raw_backward_fake(grad_logits, grad_xo, grad_regs, key, params, handle, in_shape, in_dtype):
    return grad_logits.new_empty(in_shape, dtype=_GRAD_DTYPES[in_dtype]), [torch.empty_like(p) for p in params]


def _head_raw_setup_context(ctx, inputs, output):
    t, params, handle, layer, num_registers, dtype_code, batch, hp, wp = inputs
    ctx.save_for_backward(output[3], *params)
    ctx.handle = handle
    ctx.in_shape = list(t.shape)
    ctx.in_dtype = _GRAD_DTYPES.index(t.dtype)


def _head_raw_backward_formula(ctx, grad_logits, grad_xo, grad_regs, grad_key):
    key, *params = ctx.saved_tensors
    gin, grads = torch.ops.sdpnet.train_head_raw_backward(grad_logits, grad_xo, grad_regs, key, params, ctx.handle,
                                                          ctx.in_shape, ctx.in_dtype)
    return gin, list(grads), None, None, None, None, None, None, None


train_head_raw.register_autograd(_head_raw_backward_formula, setup_context=_head_raw_setup_context)
