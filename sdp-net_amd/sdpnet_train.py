"""Training step of the SdP-Net path on the gfx950 HIP kernels (BASELINE.json configs[4];
SURVEY.md §8(f) rank 1, rows e2 / f1).

``MainModel.forward`` in training mode (``model.train()``, the reference's
``Trainer._run_batch``, training_tools.py:77-103) runs here instead of the eval fused
path.  The forward is a chain of autograd Functions, one per sub-layer (patch embed +
embedding, each ConvMixer, each EncoderLayer, the head), so DDP's bucketed gradient
all-reduce (training_tools.py:36; RCCL over xGMI) fires per layer while the backward of
the earlier layers still runs.  Every op of both directions is a HIP kernel of
libsdpnet_hip.so:

  forward   patchify + MFMA GEMM (+pos rows) | LN (rowstats + ln_apply) | depthwise conv |
            GEMM + bias | act (+ dropout) | drop-path / residual (rowscale_add) |
            attention as S = QK^T (gemm_flex) -> softmax (+ dropout) -> O = PV (gemm_flex)
  backward  dX = dY W (gemm_flex, W read transposed from LDS) | dW = dY^T X (gemm_flex,
            split-K slabs + seg_colsum) | bias / LN-affine / embedding grads (seg_colsum) |
            act' (+ the same dropout mask, regenerated from its seed) | LN backward |
            depthwise conv: input grad = conv with the flipped kernel, weight grad = dw_wgrad |
            attention: dV = Pd^T dO, dPd = dO V^T, dS = softmax', dQ = dS K, dK = dS^T Q |
            q/k head-LN backward
  loss      cross_entropy(): label-smoothed CE + dlogits in one kernel (training_tools.py:76, :88)
  optimizer AdamW: one multi-tensor kernel for GradScaler unscale + inf check +
            clip_grad_norm_ + AdamW (training_tools.py:91-99, :235), no host sync.

Randomness: dropout masks (layers.py:291, :301-308, head :450-454) come from a counter
hash of a per-op seed drawn from torch's CPU generator (so ``torch.manual_seed`` fixes a
run) and are regenerated, not stored; drop-path (StochasticDepth, utility_layers.py:16-27)
draws one Bernoulli(1-p)/(1-p) scale per sample the same way.  The reference's own RNG
stream cannot be reproduced bit for bit, so parity is pinned with dropout / drop-path
off (the reference's gradients and AdamW step as fixtures) and the masks are tested
statistically and for forward/backward consistency.

dtype: fp32 params (as the reference keeps them), compute in bf16 under
``torch.autocast("cuda", bf16)`` / bf16 inputs (the reference's training forward,
training_tools.py:85) or exact fp32 otherwise.  Gradients are fp32.  In bf16 mode the
residual stream (the token rows between sub-layers, ``x + drop_path(branch)``) and its
gradient stay fp32, as autocast keeps them: LayerNorm reads fp32 rows and writes the bf16
GEMM operand, each branch's bf16 output is added into the fp32 stream, and the stream
gradient is rounded to bf16 only where it enters a branch (``stream_dtype``;
``set_fp32_stream(False)`` gives the all-bf16 stream).
"""
from __future__ import annotations

import math
import os
import struct
from typing import List, Optional

import torch
import torch.nn as nn

import sdpnet_hip as sp
from sdpnet_engine import act_code, as_dtype, compute_dtype, f32, num_reg_rows

Rows = sp.Rows

_FP32_STREAM = os.environ.get("SDPNET_TRAIN_FP32_STREAM", "1") != "0"
# GEMM + activation fusion (sdp_gemm_train_epi): bit-identical but measured slower on the XL step
# (856 vs 890 img/s: the exact-erf GELU runs in the tile epilogue while the MFMAs idle), so off
_FUSED_EPI_MODE = os.environ.get("SDPNET_TRAIN_FUSED_EPI", "0")  # 0 off, 1 both, fwd, bwd (A/B)
_FUSED_EPI_FWD = _FUSED_EPI_MODE in ("1", "fwd")
_FUSED_EPI_BWD = _FUSED_EPI_MODE in ("1", "bwd")


def set_fp32_stream(on: bool) -> None:
    """bf16 training keeps the residual stream and its gradient in fp32 (default) or bf16."""
    global _FP32_STREAM
    _FP32_STREAM = bool(on)


def stream_dtype(dt, C: int):
    """dtype of the residual stream for compute dtype ``dt`` and width C (the mixed-dtype
    kernels take C % 8 == 0, C <= 2048)."""
    if dt == torch.bfloat16 and _FP32_STREAM and C % 8 == 0 and C <= 2048:
        return torch.float32
    return dt


def _dense(t: torch.Tensor) -> Rows:
    return Rows(t, t.shape[-1])


def _empty(shape, dt, dev):
    return torch.empty(shape, dtype=dt, device=dev)


def _seed() -> int:
    return int(torch.randint(0, 2 ** 62, (1,)).item())


class _RNG:
    """Per-forward seed source: op k of a forward gets base + k * golden (distinct streams)."""

    def __init__(self):
        self.base = _seed()
        self.k = 0

    def next(self) -> int:
        self.k += 1
        return (self.base + self.k * 0x9E3779B97F4A7C15) & 0x7FFFFFFFFFFFFFFF


def _drop_path_scale(p: float, B: int, dev) -> Optional[torch.Tensor]:
    """StochasticDepth (utility_layers.py:16-27): per-sample Bernoulli(1-p)/(1-p), or None."""
    if p <= 1e-5:
        return None
    keep = (torch.rand(B) >= p).float() / (1.0 - p)
    return keep.to(dev, non_blocking=True)


# ---------------------------------------------------------------------------
# GEMM helpers
# ---------------------------------------------------------------------------
def _linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], out_dt) -> torch.Tensor:
    """z = x . w^T + b (fast MFMA GEMM for bf16 shapes that take it, generic otherwise)."""
    M, K = x.shape
    N = w.shape[0]
    z = _empty((M, N), out_dt, x.device)
    sp.gemm(_dense(x), w, _dense(z), M, N, K, bias=b)
    return z


def _dgrad(dy: torch.Tensor, w: torch.Tensor, wt: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dx = dy . w.  Shapes the 256x256 MFMA kernel takes (bf16, N % 64 == 0, M >= 128) run on it
    with a transposed weight copy (``wt`` from the step's weight preparation, else a HIP
    transpose); others on gemm_flex, which reads w transposed from LDS."""
    M, N = dy.shape
    K = w.shape[1]
    dx = _empty((M, K), dy.dtype, dy.device)
    if sp.gemm_variant(dy.dtype, M, K, N) == 1:
        wt = wt if wt is not None else sp.transpose(w)
        sp.gemm(_dense(dy), wt, _dense(dx), M, K, N)
        return dx
    sp.gemm_flex(dy, w, dx, M, K, N, ta=False, tb=False)
    return dx


def _linear_act(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], dt, act: int, p: float = 0.0,
                seed: int = 0):
    """(z, h): z = x . w^T + b (kept for the backward), h = dropout_p(act(z)) -- one fast-kernel
    launch with a two-output epilogue when it takes the shape (bit-identical to gemm + act_fwd)."""
    M, K = x.shape
    N = w.shape[0]
    z = _empty((M, N), dt, x.device)
    h = _empty((M, N), dt, x.device)
    if _FUSED_EPI_FWD and dt == torch.bfloat16 and sp.gemm_train_epi(1, x, w, z, M, N, K, bias=b, y2=h, act=act, p=p,
                                                                seed=seed):
        return z, h
    sp.gemm(_dense(x), w, _dense(z), M, N, K, bias=b)
    sp.act_fwd(z, h, M, N, act, p, seed)
    return z, h


def _dgrad_act(dy: torch.Tensor, w: torch.Tensor, z: torch.Tensor, act: int, p: float = 0.0, seed: int = 0,
               wt: Optional[torch.Tensor] = None):
    """dz = dropout_p(dy . w) * act'(z): the input gradient through a Linear and the activation
    (+ dropout) before it, the activation backward fused into the fast kernel's epilogue when it
    takes the shape (bit-identical to _dgrad + act_bwd)."""
    M, N = dy.shape
    K = w.shape[1]
    if _FUSED_EPI_BWD and sp.gemm_variant(dy.dtype, M, K, N) == 1:
        dz = _empty((M, K), dy.dtype, dy.device)
        if sp.gemm_train_epi(2, dy, wt if wt is not None else sp.transpose(w), dz, M, K, N, z=z, act=act, p=p,
                             seed=seed):
            return dz
    dh = _dgrad(dy, w, wt)
    dz = _empty((M, K), dy.dtype, dy.device)
    sp.act_bwd(z, dh, dz, M, K, act, p, seed)
    return dz


# ---------------------------------------------------------------------------
# Per-step weight preparation: the bf16 GEMM operands of every ConvMixer / EncoderLayer weight
# (forward) and their transposes (input-gradient GEMMs) from the fp32 parameters, in ONE
# sdp_mt_cast_transpose launch at the start of a bf16 training forward, into buffers kept on
# the model.  Only valid inside that forward (_WPREP is cleared after it), so a sub-module
# trained on its own or an fp32 forward never sees them.
# ---------------------------------------------------------------------------
_WPREP: Optional[dict] = None
_WPREP_ON = os.environ.get("SDPNET_WEIGHT_PREP", "1") != "0"


def _weight_jobs(model):
    """(key, [(param, row offset in the stacked weight)], rows, cols) of every prepared weight."""
    jobs = []
    encs = [blk.t_block for blk in model.blocks] + [model.final_block.t_block]
    for blk in model.blocks:
        for mx in blk.conv_blocks:
            for conv in (mx.conv2d[1], mx.conv1d[0], mx.conv1d[2]):
                w = conv.weight
                jobs.append((id(w), [(w, 0)], w.shape[0], w.shape[1]))
    for e in encs:
        C = e.embedding_dim
        jobs.append((("qkv", id(e.q_proj.weight)), [(e.q_proj.weight, 0), (e.k_proj.weight, C), (e.v_proj.weight, 2 * C)],
                     3 * C, C))
        for lin in (e.o_proj, e.ff_linear1, e.ff_linear2):
            w = lin.weight
            jobs.append((id(w), [(w, 0)], w.shape[0], w.shape[1]))
    return jobs


def _prep_weights(model, dt) -> Optional[dict]:
    """Fill the step's bf16 weight operands (and transposes) in one launch; returns
    {key: (w [R, C] bf16, w^T [C, R] bf16)} (key = id(param), or ("qkv", id(q weight)))."""
    if not _WPREP_ON or dt != torch.bfloat16:
        return None
    dev = model.conv_init.conv.weight.device
    if dev.type != "cuda":
        return None
    jobs = _weight_jobs(model)
    sig = tuple((k, r, c, tuple((p.data_ptr(), off) for p, off in ps)) for k, ps, r, c in jobs)
    st = model.__dict__.get("_sdp_wprep")
    if st is None or st["dev"] != dev or st["shapes"] != tuple((k, r, c) for k, _, r, c in jobs):
        bufs, tiles = {}, []
        for k, ps, r, c in jobs:
            bufs[k] = (_empty((r, c), torch.bfloat16, dev), _empty((c, r), torch.bfloat16, dev))
        ei = 0
        for k, ps, r, c in jobs:
            for p, off in ps:
                pr, pc = p.shape[0], p.numel() // p.shape[0]
                for r0 in range(0, pr, 64):
                    for c0 in range(0, pc, 64):
                        tiles.append((ei, r0, c0, 0))
                ei += 1
        st = dict(dev=dev, shapes=tuple((k, r, c) for k, _, r, c in jobs), bufs=bufs, sig=None,
                  tiles=torch.tensor(tiles, dtype=torch.int32, device=dev), ntiles=len(tiles), entries=None)
        model.__dict__["_sdp_wprep"] = st
    if st["sig"] != sig:  # parameter storage moved (or first call): rebuild the entry table
        eb = sp.lib().sdp_mt_cast_transpose_entry_bytes()
        raw = bytearray()
        for k, ps, r, c in jobs:
            w, wt = st["bufs"][k]
            for p, off in ps:
                if p.dtype != torch.float32 or not p.is_contiguous():
                    return None
                pr, pc = p.shape[0], p.numel() // p.shape[0]
                ent = struct.pack("<QQQqqii", p.data_ptr(), w.data_ptr() + 2 * off * c, wt.data_ptr() + 2 * off,
                                  c, r, pr, pc)
                raw += ent + bytes(eb - len(ent))
        st["entries"] = torch.frombuffer(raw, dtype=torch.uint8).to(dev)
        st["sig"] = sig
    sp._check(sp.lib().sdp_mt_cast_transpose(st["entries"].data_ptr(), st["tiles"].data_ptr(), st["ntiles"],
                                             torch.cuda.current_stream(dev).cuda_stream), "mt_cast_transpose")
    return st["bufs"]


def _wprep(key, dt):
    """The prepared (w, w^T) of a weight inside a bf16 training forward, else None."""
    if _WPREP is None or dt != torch.bfloat16:
        return None
    return _WPREP.get(key)


_WGRAD_8PH = os.environ.get("SDPNET_WGRAD_8PH", "1") != "0"
# workgroups per weight gradient (tiles x K splits): one per CU fills the chip when the dW runs
# alone; fewer splits write fewer fp32 slabs while the dX GEMM shares the chip (A/B knob)
_WGRAD_WGS = int(os.environ.get("SDPNET_WGRAD_WGS", "256"))
# dropout of the encoder's output projections fused into the drop-path / residual pass (A/B knob)
_DMODE = 1 if os.environ.get("SDPNET_FUSED_DROPOUT", "1") != "0" else 0


def _wgrad_8ph_ok(dy: torch.Tensor, x: torch.Tensor) -> bool:
    M, N = dy.shape
    K = x.shape[1]
    return (_WGRAD_8PH and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and N % 256 == 0
            and K % 256 == 0 and M >= 256 and dy.stride(1) == 1 and x.stride(1) == 1 and dy.stride(0) % 8 == 0
            and x.stride(0) % 8 == 0 and dy.data_ptr() % 16 == 0 and x.data_ptr() % 16 == 0)


def _wgrad_8ph(dy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """dW [N, K] fp32 = dy^T x on the 8-phase MFMA kernel (csrc/wgrad.hip): the token rows are
    split into at most one workgroup per CU's worth of fp32 slabs, reduced in a fixed order by
    sdp_seg_colsum (bit-reproducible)."""
    M, N = dy.shape
    K = x.shape[1]
    nkt = -(-M // 64)
    tiles = (N // 256) * (K // 256)
    target = max(1, min(nkt, _WGRAD_WGS // tiles))
    kchunk = -(-nkt // target)
    splits = -(-nkt // kchunk)
    dw = _empty((N, K), torch.float32, dy.device)
    if splits == 1:
        sp.gemm_wgrad(dy, x, dw, M, kchunk)
    else:
        slabs = _empty((splits, N, K), torch.float32, dy.device)
        sp.gemm_wgrad(dy, x, slabs, M, kchunk, split_stride=N * K)
        sp.seg_colsum(slabs.view(splits, N * K), dw.view(1, N * K), 1, splits, 0, 1, N * K)
    return dw


# Weight-gradient work of a layer's backward (dW GEMMs, bias column sums, the depthwise weight
# gradient) is off the critical dX chain: it runs on a side stream, so its workgroups fill the
# partial tile rounds of the dX GEMMs and the memory-bound passes, and the main stream waits for it
# before the layer's backward returns (autograd / DDP hooks only ever see finished gradients).
_WSTREAM = os.environ.get("SDPNET_WGRAD_STREAM", "1") != "0"
_SIDE_STREAMS = {}


class _Side:
    def __init__(self, dev):
        self.on = _WSTREAM and dev.type == "cuda"
        if self.on:
            self.main = torch.cuda.current_stream(dev)
            key = (dev.index, self.main.cuda_stream)
            if key not in _SIDE_STREAMS:
                _SIDE_STREAMS[key] = torch.cuda.Stream(device=dev)
            self.side = _SIDE_STREAMS[key]

    def run(self, fn, *inputs):
        """fn() on the side stream after everything queued on the main stream so far; its input
        tensors are kept from reuse until the side stream has read them, its outputs until the
        main stream's work on them is done."""
        if not self.on:
            return fn()
        self.side.wait_stream(self.main)
        with torch.cuda.stream(self.side):
            out = fn()
        for t in inputs:
            if t is not None:
                t.record_stream(self.side)
        for o in (out if isinstance(out, tuple) else (out,)):
            if o is not None:
                o.record_stream(self.main)
        return out

    def join(self):
        if self.on:
            self.main.wait_stream(self.side)


def _wgrad(dy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """dW [N, K] fp32 = dy^T x, reduction over the M token rows split across workgroups."""
    if _wgrad_8ph_ok(dy, x):
        return _wgrad_8ph(dy, x)
    M, N = dy.shape
    K = x.shape[1]
    tiles = ((N + 127) // 128) * ((K + 127) // 128)
    splits = max(1, min(32, (512 + tiles - 1) // tiles, M // 512))
    if splits == 1:
        dw = _empty((N, K), torch.float32, dy.device)
        sp.gemm_flex(dy, x, dw, N, K, M, ta=True, tb=False)
        return dw
    slabs = _empty((splits, N, K), torch.float32, dy.device)
    sp.gemm_flex(dy, x, slabs, N, K, M, ta=True, tb=False, ldc=K, splits=splits, split_stride=N * K)
    dw = _empty((N, K), torch.float32, dy.device)
    sp.seg_colsum(slabs.view(splits, N * K), dw.view(1, N * K), 1, splits, 0, 1, N * K)
    return dw


def _colsum(x: torch.Tensor) -> torch.Tensor:
    """Column sums (fp32) of a [M, N] matrix: per-256-row chunk sums first (parallel over
    chunks), then the chunk sums (deterministic, no atomics)."""
    M, N = x.shape
    out = _empty((N,), torch.float32, x.device)
    full = M // 256
    if full < 4:
        sp.seg_colsum(x, out.view(1, N), 1, M, 0, 1, N)
        return out
    tail = M - full * 256
    part = _empty((full + (1 if tail else 0), N), torch.float32, x.device)
    sp.seg_colsum(x, part, full, 256, 256, 1, N)
    if tail:
        sp.seg_colsum(x, part[full:], 1, tail, 0, 1, N, x_off=full * 256 * N)
    sp.seg_colsum(part, out.view(1, N), 1, part.shape[0], 0, 1, N)
    return out


def _dense_copy(src: Rows, M: int, C: int, dt, scale: Optional[torch.Tensor] = None, sgrp: int = 1) -> torch.Tensor:
    out = _empty((M, C), dt, src.t.device)
    sp.rowscale_add(src, _dense(out), M, C, scale=scale, sgrp=sgrp)
    return out


def _branch_grad(d: torch.Tensor, T: int, C: int, dt, dp: Optional[torch.Tensor], grp: int, p: float, seed: int):
    """Gradient into a residual branch y = x + drop_path(dropout(z)): dz = d * mask / (1-p) * dp
    (one pass; no copy at all when neither is active and d is already in the branch dtype).
    An fp32 stream gradient is rounded to the bf16 branch first (with the drop-path scale),
    then the dropout mask is applied in place."""
    if d.dtype != dt:
        out = _empty((T, C), dt, d.device)
        # one pass: cast (with the drop-path scale), then the dropout mask on the rounded value
        if _DMODE:
            sp.rowscale_add(_dense(d), _dense(out), T, C, scale=dp, sgrp=grp, p=p, seed=seed, dmode=2)
        else:
            sp.rowscale_add(_dense(d), _dense(out), T, C, scale=dp, sgrp=grp)
            if p > 0:
                sp.act_bwd(out, out, out, T, C, 0, p, seed)
        return out
    if p <= 0 and dp is None:
        return d
    out = _empty((T, C), dt, d.device)
    if not _DMODE and p > 0:
        sp.act_bwd(d, d, out, T, C, 0, p, seed)
        d = out
    sp.rowscale_add(_dense(d), _dense(out), T, C, scale=dp, sgrp=grp, p=p, seed=seed, dmode=_DMODE)
    return out


# SDPNET_TRAIN_REG_FOLD=0: the ConvMixer's register-row copies as separate launches (A/B switch)
_REG_FOLD = os.environ.get("SDPNET_TRAIN_REG_FOLD", "1") != "0"


def _regs(src: torch.Tensor, dsts, B: int, R: int, N: int):
    """The register-row copy job src -> dsts for a row kernel to fold in (None: nothing left to copy)."""
    if not R:
        return None
    if not _REG_FOLD:
        sp.copy_regs((src, dsts, B, R, N))
        return None
    return (src, dsts, B, R, N)


def _add_ln_fwd(x: Rows, y: Rows, M: int, C: int, resid: Rows, g: torch.Tensor, b: torch.Tensor, eps: float, dt,
                scale=None, sgrp: int = 1, act: int = 0, p: float = 0.0, seed: int = 0, dmode: int = 0, regs=None):
    """y = act / dropout(x) * scale + resid (the branch add), then (a, stats) = LN(y): one pass
    (sp.add_ln_fwd) where it applies, else rowscale_add + _ln_fwd (bit-identical either way); regs: a
    register-row copy job (sp.add_ln_fwd) done in the same launch."""
    st = _empty((M, 2), torch.float32, x.t.device)
    a = _empty((M, C), dt, x.t.device)
    if _ADD_LN and sp.add_ln_fwd(x, y, _dense(a), M, C, resid, eps, g, b, st, scale=scale, sgrp=sgrp, act=act, p=p,
                                 seed=seed, dmode=dmode, regs=regs):
        return a, st
    sp.copy_regs(regs)
    sp.rowscale_add(x, y, M, C, scale=scale, sgrp=sgrp, resid=resid, act=act, p=p, seed=seed, dmode=dmode)
    return _ln_fwd(y, M, C, g, b, eps, dt)


# SDPNET_TRAIN_ADD_LN=0: the branch add and the next LayerNorm as two passes (A/B switch)
_ADD_LN = os.environ.get("SDPNET_TRAIN_ADD_LN", "1") != "0"
# SDPNET_TRAIN_LN_EMIT=0: the branch gradient after a LayerNorm backward as separate passes (A/B switch)
_LN_EMIT = os.environ.get("SDPNET_TRAIN_LN_EMIT", "1") != "0"


def _ln_fwd(x: Rows, M: int, C: int, g: torch.Tensor, b: torch.Tensor, eps: float, dt):
    st = _empty((M, 2), torch.float32, x.t.device)
    a = _empty((M, C), dt, x.t.device)
    if C % 8 == 0 and C <= 2048 and x.ld % 8 == 0:
        sp.ln_fwd(x, eps, g, b, st, _dense(a), M, C)      # one pass: stats + normalized rows
    else:
        sp.rowstats(x, eps, st, M, C)
        sp.ln_apply(x, st, g, b, _dense(a), M, C)
    return a, st


# ---------------------------------------------------------------------------
# ConvMixer (layers.py:63-104)
# ---------------------------------------------------------------------------
def _mixer_params(m) -> List[Optional[nn.Parameter]]:
    dw, cc, up, dn = m.conv2d[0], m.conv2d[1], m.conv1d[0], m.conv1d[2]
    return [m.layer_norm_1.gamma, m.layer_norm_1.beta, dw.weight, dw.bias, cc.weight, cc.bias,
            m.layer_norm_2.gamma, m.layer_norm_2.beta, up.weight, up.bias, dn.weight, dn.bias]


# set by eval_forward: the training forward's kernels without dropout / drop path (eval semantics)
_NO_DROP = False


def _drop_p(module) -> float:
    if _NO_DROP:
        return 0.0
    return float(module.p) if hasattr(module, "p") else 0.0


class _MixerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tok, geo, m, dt, *params):
        B, R, H, W = geo
        g1, b1, dww, dwb, ccw, ccb, g2, b2, upw, upb, dnw, dnb = params
        C = ccw.shape[0]
        P, N = H * W, R + H * W
        M = B * P
        k = dww.shape[-1]
        dev = tok.device
        act = act_code(m.activation)
        img = Rows(tok, C, P, N, R)
        pcc, pup, pdn = _wprep(id(ccw), dt), _wprep(id(upw), dt), _wprep(id(dnw), dt)
        W_ = dict(g1=f32(g1), b1=f32(b1), dww=f32(dww.reshape(C, k * k)), dwb=f32(dwb),
                  ccw=pcc[0] if pcc else as_dtype(ccw.reshape(C, C), dt), ccb=f32(ccb), g2=f32(g2), b2=f32(b2),
                  upw=pup[0] if pup else as_dtype(upw.reshape(4 * C, C), dt), upb=f32(upb),
                  dnw=pdn[0] if pdn else as_dtype(dnw.reshape(C, 4 * C), dt), dnb=f32(dnb),
                  ccw_t=pcc[1] if pcc else None, upw_t=pup[1] if pup else None, dnw_t=pdn[1] if pdn else None)
        dp2 = _drop_path_scale(_drop_p(m.drop_path_2), B, dev)
        dp1 = _drop_path_scale(_drop_p(m.drop_path_1), B, dev)
        # x_ = drop_path_2(act(PW(DW(LN1 x)))) + x
        a1, s1 = _ln_fwd(img, M, C, W_["g1"], W_["b1"], m.layer_norm_1.eps, dt)
        d = _empty((M, C), dt, dev)
        sp.dwconv(_dense(a1), W_["dww"], W_["dwb"], _dense(d), B, H, W, C, k)
        z1 = _linear(d, W_["ccw"], W_["ccb"], dt)
        mid = torch.empty_like(tok)
        out = torch.empty_like(tok)
        imid = Rows(mid, C, P, N, R)
        # act + drop path + residual, then LN2 of the sum (one pass; the register rows of mid and out
        # copied from tok by the same launch)
        # x = drop_path_1(PW_down(act(PW_up(LN2 x_)))) + x_
        a2, s2 = _add_ln_fwd(_dense(z1), imid, M, C, img, W_["g2"], W_["b2"], m.layer_norm_2.eps, dt, scale=dp2, sgrp=P,
                             act=act, regs=_regs(tok, [mid, out], B, R, N))
        z2, h = _linear_act(a2, W_["upw"], W_["upb"], dt, act)
        if dp1 is None and tok.dtype == dt:  # residual add in the GEMM epilogue, straight into the token rows
            sp.gemm(_dense(h), W_["dnw"], Rows(out, C, P, N, R), M, C, 4 * C, bias=W_["dnb"], resid=imid)
        else:
            z3 = _linear(h, W_["dnw"], W_["dnb"], dt)
            sp.rowscale_add(_dense(z3), Rows(out, C, P, N, R), M, C, scale=dp1, sgrp=P, resid=imid)
        ctx.st = dict(tok=tok, mid=mid, a1=a1, s1=s1, d=d, z1=z1, a2=a2, s2=s2, z2=z2, h=h, W=W_, dp1=dp1, dp2=dp2,
                      geo=(B, R, H, W, C, k), act=act, dt=dt, has=[p is not None for p in params])
        ctx.shapes = [None if p is None else p.shape for p in params]
        return out

    @staticmethod
    def backward(ctx, dout):
        S = ctx.st
        B, R, H, W, C, k = S["geo"]
        P, N = H * W, R + H * W
        M = B * P
        dt, act, W_ = S["dt"], S["act"], S["W"]
        dout = dout.contiguous().to(S["tok"].dtype)  # stream dtype
        dev = dout.device
        iout = Rows(dout, C, P, N, R)
        # branch 1
        dz3 = _dense_copy(iout, M, C, dt, S["dp1"], P)
        dz2 = _dgrad_act(dz3, W_["dnw"], S["z2"], act, wt=W_["dnw_t"])
        has = S["has"]  # [g1, b1, dww, dwb, ccw, ccb, g2, b2, upw, upb, dnw, dnb]: bias grads only if the bias exists
        side = _Side(dev)
        h_, a2_, d_, a1_ = S["h"], S["a2"], S["d"], S["a1"]
        gdn, gdnb = side.run(lambda: (_wgrad(dz3, h_), _colsum(dz3) if has[11] else None), dz3, h_)
        da2 = _dgrad(dz2, W_["upw"], W_["upw_t"])
        gup, gupb = side.run(lambda: (_wgrad(dz2, a2_), _colsum(dz2) if has[9] else None), dz2, a2_)
        dmid = torch.empty_like(dout)  # register rows copied from dout by the LN2 backward's launch
        regs = _regs(dout, [dmid], B, R, N)
        imid = Rows(dmid, C, P, N, R)
        dz1 = _empty((M, C), dt, dev)
        if _LN_EMIT and dt == torch.bfloat16:  # branch 2's gradient dz1 written by the LN2 backward
            gg2, gb2 = sp.ln_bwd(Rows(S["mid"], C, P, N, R), S["s2"], W_["g2"], _dense(da2), imid, M, C, add=iout,
                                 emit=dict(out=dz1, scale=S["dp2"], sgrp=P, z=S["z1"], act=act), regs=regs)
        else:
            gg2, gb2 = sp.ln_bwd(Rows(S["mid"], C, P, N, R), S["s2"], W_["g2"], _dense(da2), imid, M, C, add=iout,
                                 regs=regs)
            # branch 2
            dh1 = _dense_copy(imid, M, C, dt, S["dp2"], P)
            sp.act_bwd(S["z1"], dh1, dz1, M, C, act)
        dd = _dgrad(dz1, W_["ccw"], W_["ccw_t"])
        gcc, gccb = side.run(lambda: (_wgrad(dz1, d_), _colsum(dz1) if has[5] else None), dz1, d_)
        da1 = _empty((M, C), dt, dev)
        wflip = W_["dww"].view(C, k, k).flip(1, 2).reshape(C, k * k).contiguous()
        sp.dwconv(_dense(dd), wflip, None, _dense(da1), B, H, W, C, k)
        gdw, gdwb = side.run(lambda: (sp.dw_wgrad(_dense(a1_), _dense(dd), B, H, W, C, k),
                                      _colsum(dd) if has[3] else None), a1_, dd)
        dx = dmid  # residual; LN1's input gradient is added in place on the image rows
        idx = Rows(dx, C, P, N, R)
        gg1, gb1 = sp.ln_bwd(Rows(S["tok"], C, P, N, R), S["s1"], W_["g1"], _dense(da1), idx, M, C, add=idx)
        grads = [gg1, gb1, gdw, gdwb, gcc, gccb, gg2, gb2, gup, gupb, gdn, gdnb]
        side.join()
        ctx.st = None
        return (dx, None, None, None, *[g.view(shp) if h else None for g, shp, h in zip(grads, ctx.shapes, S["has"])])


# ---------------------------------------------------------------------------
# EncoderLayer (layers.py:215-316)
# ---------------------------------------------------------------------------
def _enc_params(e) -> List[Optional[nn.Parameter]]:
    qn = isinstance(e.q_norm, nn.LayerNorm)
    return [e.norm1.weight, e.norm1.bias, e.q_proj.weight, e.k_proj.weight, e.v_proj.weight,
            e.q_norm.weight if qn else None, e.q_norm.bias if qn else None,
            e.k_norm.weight if qn else None, e.k_norm.bias if qn else None,
            e.o_proj.weight, e.norm2.weight, e.norm2.bias, e.ff_linear1.weight, e.ff_linear1.bias,
            e.ff_linear2.weight, e.ff_linear2.bias]


def _attn_materialized(qkvn, B, N, C, Hn, hd, Np, Z, dt, dev, p_att, seed, mask=None):
    """Attention with S / P materialised per (b, h) (fp32 path, and shapes the flash kernels
    do not take): S = QK^T (fp32) -> softmax (+ dropout) -> O = Pd V.  ``qkvn`` is the fp32
    operand copy in bf16 mode (P, dP and dS then stay fp32 as in the flash kernels; O is
    rounded to dt)."""
    T = B * N
    adt = qkvn.dtype
    Sm = _empty((B, Hn, N, Np), torch.float32, dev)
    sp.gemm_flex(qkvn, qkvn, Sm, N, N, hd, ta=False, tb=True, lda=3 * C, ldb=3 * C, ldc=Np, Z=Z, zdiv=Hn,
                 sa=(N * 3 * C, hd), sb=(N * 3 * C, hd), sc=(Hn * N * Np, N * Np), b_off=C)
    Pm = _empty((B, Hn, N, Np), adt, dev)
    Pd = _empty((B, Hn, N, Np), adt, dev) if p_att > 0 else Pm
    sp.softmax_fwd(Sm.view(-1, Np), Pm.view(-1, Np), Pd.view(-1, Np) if p_att > 0 else None, Z * N, N, Np,
                   1.0 / math.sqrt(hd), p_att, seed, mask=mask)
    del Sm
    o = _empty((T, C), adt, dev)
    sp.gemm_flex(Pd, qkvn, o, N, hd, N, ta=False, tb=False, lda=Np, ldb=3 * C, ldc=C, Z=Z, zdiv=Hn,
                 sa=(Hn * N * Np, N * Np), sb=(N * 3 * C, hd), sc=(N * C, hd), b_off=2 * C)
    return (o if adt == dt else sp.cast(o, dt)), None, Pm, Pd


def _attn_materialized_bwd(qkvn, Pm, Pd, do, dqkv, dqk, B, N, C, Hn, hd, Np, Z, dt, dev, p_att, seed):
    adt = qkvn.dtype
    if do.dtype != adt:
        do = sp.cast(do, adt)
    dPd = _empty((B, Hn, N, Np), adt, dev)
    sp.gemm_flex(do, qkvn, dPd, N, N, hd, ta=False, tb=True, lda=C, ldb=3 * C, ldc=Np, Z=Z, zdiv=Hn,
                 sa=(N * C, hd), sb=(N * 3 * C, hd), sc=(Hn * N * Np, N * Np), b_off=2 * C)
    sp.gemm_flex(Pd, do, dqkv, N, hd, N, ta=True, tb=False, lda=Np, ldb=C, ldc=3 * C, Z=Z, zdiv=Hn,
                 sa=(Hn * N * Np, N * Np), sb=(N * C, hd), sc=(N * 3 * C, hd), c_off=2 * C)      # dV
    dS = _empty((B, Hn, N, Np), adt, dev)
    sp.softmax_bwd(Pm.view(-1, Np), dPd.view(-1, Np), dS.view(-1, Np), Z * N, N, Np, p_att, seed)
    del dPd
    scale = 1.0 / math.sqrt(hd)
    sp.gemm_flex(dS, qkvn, dqk, N, hd, N, ta=False, tb=False, lda=Np, ldb=3 * C, ldc=3 * C, Z=Z, zdiv=Hn,
                 sa=(Hn * N * Np, N * Np), sb=(N * 3 * C, hd), sc=(N * 3 * C, hd), b_off=C, alpha=scale)   # dQ
    sp.gemm_flex(dS, qkvn, dqk, N, hd, N, ta=True, tb=False, lda=Np, ldb=3 * C, ldc=3 * C, Z=Z, zdiv=Hn,
                 sa=(Hn * N * Np, N * Np), sb=(N * 3 * C, hd), sc=(N * 3 * C, hd), c_off=C, alpha=scale)   # dK


class _EncoderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tok, geo, e, dt, rng, *params):
        B, N = geo[:2]
        mask = geo[2] if len(geo) > 2 else None  # additive bias (EncoderLayer._mask_bias) + strides
        (n1g, n1b, wq, wk, wv, qg, qb, kg, kb, wo, n2g, n2b, w1, b1, w2, b2) = params
        C, Hn, hd = e.embedding_dim, e.n_head, e.head_dim
        T = B * N
        dev = tok.device
        act = act_code(e.activation)
        p_ff = 0.0 if _NO_DROP else float(e.dropout.p)
        p_att = float(e.att_dropout) if e.fast_att and not _NO_DROP else p_ff  # manual path drops with self.dropout (:297)
        qn = qg is not None
        pq, po, p1, p2 = _wprep(("qkv", id(wq)), dt), _wprep(id(wo), dt), _wprep(id(w1), dt), _wprep(id(w2), dt)
        wqkv = pq[0] if pq else as_dtype(torch.cat([f32(wq), f32(wk), f32(wv)], 0), dt)
        W_ = dict(n1g=f32(n1g), n1b=f32(n1b), wqkv=wqkv, wo=po[0] if po else as_dtype(wo, dt), n2g=f32(n2g),
                  n2b=f32(n2b), w1=p1[0] if p1 else as_dtype(w1, dt), b1=f32(b1), w2=p2[0] if p2 else as_dtype(w2, dt),
                  b2=f32(b2), wqkv_t=pq[1] if pq else None, wo_t=po[1] if po else None, w1_t=p1[1] if p1 else None,
                  w2_t=p2[1] if p2 else None)
        if qn:
            W_.update(qg=f32(qg), qb=f32(qb), kg=f32(kg), kb=f32(kb))
        seeds = [rng.next() for _ in range(4)]
        dp1 = _drop_path_scale(_drop_p(e.drop_path1), B, dev)
        dp2 = _drop_path_scale(_drop_p(e.drop_path2), B, dev)
        a1, s1 = _ln_fwd(_dense(tok), T, C, W_["n1g"], W_["n1b"], e.norm1.eps, dt)
        qkv = _linear(a1, W_["wqkv"], None, dt)                          # :282-284
        qkvn, sq, sk = qkv, None, None
        if qn:                                                          # :286
            qkvn = _empty((T, 3 * C), dt, dev)
            sp.copy_rows(qkv[:, 2 * C:], 3 * C, 0, qkvn[:, 2 * C:], 3 * C, 0, 1, T, C)  # v third
            rq = Rows(qkv, hd, Hn, 3 * Hn, 0)
            rk = Rows(qkv, hd, Hn, 3 * Hn, Hn)
            sq = _empty((T * Hn, 2), torch.float32, dev)
            sk = _empty((T * Hn, 2), torch.float32, dev)
            if hd % 8 == 0:  # one pass, several heads per wave (ln_fwd_sm)
                sp.ln_fwd(rq, e.q_norm.eps, W_["qg"], W_["qb"], sq, Rows(qkvn, hd, Hn, 3 * Hn, 0), T * Hn, hd)
                sp.ln_fwd(rk, e.k_norm.eps, W_["kg"], W_["kb"], sk, Rows(qkvn, hd, Hn, 3 * Hn, Hn), T * Hn, hd)
            else:
                sp.rowstats(rq, e.q_norm.eps, sq, T * Hn, hd)
                sp.rowstats(rk, e.k_norm.eps, sk, T * Hn, hd)
                sp.ln_apply(rq, sq, W_["qg"], W_["qb"], Rows(qkvn, hd, Hn, 3 * Hn, 0), T * Hn, hd)
                sp.ln_apply(rk, sk, W_["kg"], W_["kb"], Rows(qkvn, hd, Hn, 3 * Hn, Hn), T * Hn, hd)
        # attention (:289-298): S = QK^T, P = softmax(S / sqrt(hd)), Pd = dropout(P), O = Pd V
        Np = (N + 7) // 8 * 8
        Z = B * Hn
        if mask is None and sp.attn_train_applies(dt, N, hd):  # flash form: saves O and the row LSE only
            o = _empty((T, C), dt, dev)
            lse = _empty((Z * N,), torch.float32, dev)
            sp.attn_train_fwd(qkvn, o, lse, B, N, Hn, hd, 1.0 / math.sqrt(hd), p_att, seeds[0])
            Pm = Pd = None
        else:  # masked attention, fp32, or head dims the flash kernels do not take (bf16: operands cast to
            # fp32 once; the mask enters the materialised softmax)
            qkva = qkvn if dt == torch.float32 else sp.cast(qkvn, torch.float32)
            mk = None if mask is None else (mask[0], mask[1], mask[2], Hn)
            o, lse, Pm, Pd = _attn_materialized(qkva, B, N, C, Hn, hd, Np, Z, dt, dev, p_att, seeds[0], mask=mk)

        # x = x + drop_path1(dropout(o_proj(o)))                       (:300-303)
        zo = _linear(o, W_["wo"], None, dt)
        t2 = _empty((T, C), tok.dtype, dev)                               # stream dtype
        if not _DMODE and p_ff > 0:
            sp.act_fwd(zo, zo, T, C, 0, p_ff, seeds[1])
        # dropout + drop path + residual, then LN2 of the sum (one pass)
        # x = x + drop_path2(dropout(ff2(dropout(act(ff1(LN2 x))))))   (:306-309)
        a2, s2 = _add_ln_fwd(_dense(zo), _dense(t2), T, C, _dense(tok), W_["n2g"], W_["n2b"], e.norm2.eps, dt,
                             scale=dp1, sgrp=N, p=p_ff, seed=seeds[1], dmode=_DMODE)
        del zo
        z1, h = _linear_act(a2, W_["w1"], W_["b1"], dt, act, p_ff, seeds[2])
        z2 = _linear(h, W_["w2"], W_["b2"], dt)
        out = _empty((T, C), tok.dtype, dev)
        if not _DMODE and p_ff > 0:
            sp.act_fwd(z2, z2, T, C, 0, p_ff, seeds[3])
        sp.rowscale_add(_dense(z2), _dense(out), T, C, scale=dp2, sgrp=N, resid=_dense(t2), p=p_ff, seed=seeds[3],
                        dmode=_DMODE)
        ctx.st = dict(tok=tok, a1=a1, s1=s1, qkv=qkv, qkvn=qkvn, sq=sq, sk=sk, P=Pm, Pd=Pd, lse=lse, o=o, t2=t2, a2=a2, s2=s2,
                      z1=z1, h=h, W=W_, seeds=seeds, dp1=dp1, dp2=dp2, geo=(B, N, C, Hn, hd, Np), act=act, dt=dt,
                      p_ff=p_ff, p_att=p_att, qn=qn)
        ctx.has = [p is not None for p in params]
        return out

    @staticmethod
    def backward(ctx, dout):
        S = ctx.st
        B, N, C, Hn, hd, Np = S["geo"]
        T, Z = B * N, B * Hn
        dt, act, W_, seeds = S["dt"], S["act"], S["W"], S["seeds"]
        p_ff, p_att = S["p_ff"], S["p_att"]
        sdt = S["tok"].dtype
        dout = dout.contiguous().to(sdt)
        dev = dout.device
        # FFN branch
        dz2 = _branch_grad(dout, T, C, dt, S["dp2"], N, p_ff, seeds[3])
        dz1 = _dgrad_act(dz2, W_["w2"], S["z1"], act, p_ff, seeds[2], wt=W_["w2_t"])
        side = _Side(dev)
        h_, a2_, o_, a1_ = S["h"], S["a2"], S["o"], S["a1"]
        gw2, gb2 = side.run(lambda: (_wgrad(dz2, h_), _colsum(dz2)), dz2, h_)
        da2 = _dgrad(dz1, W_["w1"], W_["w1_t"])
        gw1, gb1 = side.run(lambda: (_wgrad(dz1, a2_), _colsum(dz1)), dz1, a2_)
        dt2 = _empty((T, C), sdt, dev)
        if _LN_EMIT and _DMODE and sdt != dt and dt == torch.bfloat16:  # the attention branch's gradient from norm2's backward
            dzo = _empty((T, C), dt, dev)
            gn2g, gn2b = sp.ln_bwd(_dense(S["t2"]), S["s2"], W_["n2g"], _dense(da2), _dense(dt2), T, C, add=_dense(dout),
                                   emit=dict(out=dzo, scale=S["dp1"], sgrp=N, p=p_ff, seed=seeds[1], dmode=2))
        else:
            gn2g, gn2b = sp.ln_bwd(_dense(S["t2"]), S["s2"], W_["n2g"], _dense(da2), _dense(dt2), T, C,
                                   add=_dense(dout))
            # attention branch
            dzo = _branch_grad(dt2, T, C, dt, S["dp1"], N, p_ff, seeds[1])
        do = _dgrad(dzo, W_["wo"], W_["wo_t"])
        gwo = side.run(lambda: _wgrad(dzo, o_), dzo, o_)
        qkvn, Pm, Pd = S["qkvn"], S["P"], S["Pd"]
        scale = 1.0 / math.sqrt(hd)
        # dQ / dK land in dqk, dV in dqkv (the same buffer unless the q/k head LayerNorm follows)
        adt = dt if Pm is None else Pm.dtype
        dqkv = _empty((T, 3 * C), adt, dev)
        dqk = dqkv if not S["qn"] else _empty((T, 3 * C), adt, dev)
        if Pm is None:  # flash backward: P recomputed from Q, K and the saved LSE
            delta = _empty((Z * N,), torch.float32, dev)
            sp.attn_train_bwd(qkvn, S["o"], do, S["lse"], delta, (dqk, 0), (dqk, C), (dqkv, 2 * C), B, N, Hn, hd,
                              scale, p_att, seeds[0])
        else:
            qkva = qkvn if adt == dt else sp.cast(qkvn, adt)
            _attn_materialized_bwd(qkva, Pm, Pd, do, dqkv, dqk, B, N, C, Hn, hd, Np, Z, dt, dev, p_att, seeds[0])
            if adt != dt:  # fp32 attention internals of bf16 mode: round the q/k/v gradients once
                dqk = sp.cast(dqk, dt)
                dqkv = dqk if not S["qn"] else sp.cast(dqkv, dt)
        gqg = gqb = gkg = gkb = None
        if S["qn"]:
            qkv = S["qkv"]
            gqg, gqb = sp.ln_bwd(Rows(qkv, hd, Hn, 3 * Hn, 0), S["sq"], W_["qg"], Rows(dqk, hd, Hn, 3 * Hn, 0),
                                 Rows(dqkv, hd, Hn, 3 * Hn, 0), T * Hn, hd)
            gkg, gkb = sp.ln_bwd(Rows(qkv, hd, Hn, 3 * Hn, Hn), S["sk"], W_["kg"], Rows(dqk, hd, Hn, 3 * Hn, Hn),
                                 Rows(dqkv, hd, Hn, 3 * Hn, Hn), T * Hn, hd)
        da1 = _dgrad(dqkv, W_["wqkv"], W_["wqkv_t"])
        gqkv = side.run(lambda: _wgrad(dqkv, a1_), dqkv, a1_)
        # dzo may BE dt2 (no dropout / drop path): with the side stream still reading it, the LN
        # backward adds into a fresh buffer instead of updating dt2 in place
        dx = _empty((T, C), sdt, dev) if side.on else dt2
        gn1g, gn1b = sp.ln_bwd(_dense(S["tok"]), S["s1"], W_["n1g"], _dense(da1), _dense(dx), T, C, add=_dense(dt2))
        grads = [gn1g, gn1b, gqkv[:C], gqkv[C:2 * C], gqkv[2 * C:], gqg, gqb, gkg, gkb, gwo, gn2g, gn2b, gw1, gb1,
                 gw2, gb2]
        side.join()
        has = ctx.has
        ctx.st = None
        return (dx, None, None, None, None, *[g if h else None for g, h in zip(grads, has)])


# ---------------------------------------------------------------------------
# Patch embedding + positional / register embedding (layers.py:28-42, :116-209)
# ---------------------------------------------------------------------------
class _EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, geo, model, dt, wp, eh, ew, ereg):
        B, R, Hp, Wp, nreg_arg, sdt = geo
        pat = model.conv_init
        emb = model.embedding_layer
        C = wp.shape[0]
        p = pat.patch_size
        P, N = Hp * Wp, R + Hp * Wp
        dev = x.device
        act = act_code(emb.activation)  # layers.py:168 / :209: activation(x + pos) on the image rows
        kp = pat._kpad()
        patches = _empty((B * P, kp), dt, dev)
        sp.patchify(x.contiguous(), patches, p, kp)
        w = as_dtype(wp.reshape(C, -1), dt)
        if kp != w.shape[1]:
            wpad = torch.zeros(C, kp, dtype=dt, device=dev)
            wpad[:, : w.shape[1]].copy_(w)
            w = wpad
        conv_emb = eh is None
        if conv_emb:  # ConvEmbedding: fixed avg-pooled bone table (a buffer)
            pos = emb._pos_table(Hp, Wp)
        else:
            pos = _empty((P, C), torch.float32, dev)
            sp.pos_table(f32(eh), f32(ew), pos, Hp, Wp, C)
        tok = _empty((B * N, C), sdt, dev)
        z = None
        if sdt != dt:  # fp32 stream: tok = act(bf16(patches . w^T) + pos) in fp32 (autocast's promotion)
            zc = _linear(patches, w, None, dt)
            if act == 0:
                sp.rowscale_add(_dense(zc), Rows(tok, C, P, N, R), B * P, C, resid=Rows(pos, C, P, 0, 0))
            else:
                z = _empty((B * P, C), sdt, dev)
                sp.rowscale_add(_dense(zc), _dense(z), B * P, C, resid=Rows(pos, C, P, 0, 0))
                sp.rowscale_add(_dense(z), Rows(tok, C, P, N, R), B * P, C, act=act)
            del zc
        elif act == 0:
            posd = pos if dt == torch.float32 else as_dtype(pos, dt)
            sp.gemm(_dense(patches), w, Rows(tok, C, P, N, R), B * P, C, kp, resid=Rows(posd, C, P, 0, 0),
                    resid_pre=True)
        else:  # keep the pre-activation for the backward
            posd = pos if dt == torch.float32 else as_dtype(pos, dt)
            z = _empty((B * P, C), dt, dev)
            sp.gemm(_dense(patches), w, _dense(z), B * P, C, kp, resid=Rows(posd, C, P, 0, 0), resid_pre=True)
            sp.rowscale_add(_dense(z), Rows(tok, C, P, N, R), B * P, C, act=act)
        table, R2 = emb._register_rows(nreg_arg)
        if R:
            sp.copy_rows(table.contiguous(), C, 0, tok, C, N * C, B, R, C)
        # the image gradient (an input that requires grad, e.g. input-gradient attacks) needs w and the
        # image geometry (the compiled per-layer path passes need_dx to layer 0's op)
        need_dx = bool(getattr(ctx, "needs_input_grad", (False,))[0])
        ctx.st = dict(patches=patches, geo=(B, R, Hp, Wp, C, P, N, p, kp), dt=dt, sdt=sdt, conv_emb=conv_emb, act=act, z=z,
                      nrow_eh=None if conv_emb else eh.shape[0], nrow_ew=None if conv_emb else ew.shape[0],
                      nreg=ereg.shape[0], wshape=wp.shape, w=w if need_dx else None, img=(x.shape, x.dtype))
        return tok

    @staticmethod
    def backward(ctx, dtok):
        S = ctx.st
        B, R, Hp, Wp, C, P, N, p, kp = S["geo"]
        dt, sdt = S["dt"], S["sdt"]
        dtok = dtok.contiguous().to(sdt)
        dev = dtok.device
        dimg = _dense_copy(Rows(dtok, C, P, N, R), B * P, C, sdt)  # image rows, stream dtype
        if S["act"]:  # through the embedding activation: dz = act'(z) * d
            sp.act_bwd(S["z"], dimg, dimg, B * P, C, S["act"])
        dconv = dimg if sdt == dt else _dense_copy(_dense(dimg), B * P, C, dt)
        gw = _wgrad(dconv, S["patches"])[:, : 3 * p * p].contiguous().view(S["wshape"])
        dx = None
        if S["w"] is not None:  # the patch conv's input gradient: dpatches = dconv . W, then col2im
            dx = _empty(S["img"][0], S["img"][1], dev)
            sp.unpatchify(_dgrad(dconv, S["w"]), dx, p, kp)
        geh = gew = None
        if not S["conv_emb"]:
            dpos = _empty((P, C), torch.float32, dev)
            sp.seg_colsum(dimg, dpos, P, B, 1, P, C)                       # sum over the batch
            geh = torch.zeros(S["nrow_eh"], C, dtype=torch.float32, device=dev)
            gew = torch.zeros(S["nrow_ew"], C, dtype=torch.float32, device=dev)
            sp.seg_colsum(dpos, geh, Hp, Wp, Wp, 1, C)                      # Eh indexed by h (rows)
            sp.seg_colsum(dpos, gew, Wp, Hp, 1, Wp, C)                      # Ew indexed by w (columns)
        greg = torch.zeros(S["nreg"], C, dtype=torch.float32, device=dev)
        if R:
            off = 1 if S["conv_emb"] else 0  # ConvEmbedding takes Embedding rows 1..R (layers.py:206)
            sp.seg_colsum(dtok, greg[off:], R, B, 1, N, C)
        ctx.st = None
        return dx, None, None, None, gw, geh, gew, greg


# ---------------------------------------------------------------------------
# ClassificationHead (layers.py:429-465)
# ---------------------------------------------------------------------------
class _HeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tok, geo, head, dt, rng, *params):
        B, R, P, N, C = geo
        ln_g, ln_b, w1, b1, w2, b2 = params
        dev = tok.device
        from_reg = head.from_register
        rows, grp_off = (R, 0) if from_reg else (P, R)
        # the mean stays in the stream dtype when a LayerNorm follows (it rounds to dt itself)
        m = _empty((B, C), tok.dtype if ln_g is not None else dt, dev)
        sp.group_mean(Rows(tok, C, rows, N, grp_off), m, B, rows, C)
        st = dict(geo=geo, dt=dt, sdt=tok.dtype, from_reg=from_reg, rows=rows, off=grp_off, m=m)
        x = m
        if ln_g is not None:
            a, s = _ln_fwd(_dense(m), B, C, f32(ln_g), f32(ln_b), head.output_head[0].eps, dt)
            st.update(a=a, s=s, lng=f32(ln_g))
            x = a
        W1 = as_dtype(w1, dt)
        z1 = _linear(x, W1, f32(b1), dt)
        st.update(x=x, W1=W1)
        if w2 is None:
            ctx.st, ctx.has = st, [p is not None for p in params]
            return z1
        drop = [mm for mm in head.output_head if isinstance(mm, nn.Dropout)]
        pd = float(drop[0].p) if drop and not _NO_DROP else 0.0
        seed = rng.next()
        hh = _empty(z1.shape, dt, dev)
        sp.act_fwd(z1, hh, B, z1.shape[1], sp.ACT_CODES["tanh"], pd, seed)
        W2 = as_dtype(w2, dt)
        logits = _linear(hh, W2, f32(b2), dt)
        st.update(z1=z1, h=hh, W2=W2, pd=pd, seed=seed)
        ctx.st, ctx.has = st, [p is not None for p in params]
        return logits

    @staticmethod
    def backward(ctx, dlog):
        S = ctx.st
        B, R, P, N, C = S["geo"]
        dt = S["dt"]
        dlog = dlog.contiguous().to(dt)
        dev = dlog.device
        gw2 = gb2 = None
        if "W2" in S:
            dh = _dgrad(dlog, S["W2"])
            gw2, gb2 = _wgrad(dlog, S["h"]), _colsum(dlog)
            dz1 = _empty(dh.shape, dt, dev)
            sp.act_bwd(S["z1"], dh, dz1, B, dh.shape[1], sp.ACT_CODES["tanh"], S["pd"], S["seed"])
        else:
            dz1 = dlog
        dxh = _dgrad(dz1, S["W1"])
        gw1, gb1 = _wgrad(dz1, S["x"]), _colsum(dz1)
        glg = glb = None
        if "a" in S:
            dm = _empty((B, C), S["m"].dtype, dev)
            glg, glb = sp.ln_bwd(_dense(S["m"]), S["s"], S["lng"], _dense(dxh), _dense(dm), B, C)
        else:
            dm = dxh
        dtok = torch.zeros(B * N, C, dtype=S["sdt"], device=dev)
        rows = S["rows"]
        sp.copy_rows(dm, 0, C, dtok, C, N * C, B, rows, C, dst_offset_rows=S["off"])   # broadcast to the group
        inv = torch.full((B * rows,), 1.0 / rows, dtype=torch.float32, device=dev)
        grp = Rows(dtok, C, rows, N, S["off"])
        sp.rowscale_add(grp, grp, B * rows, C, scale=inv, sgrp=1)                        # d mean = dm / rows
        grads = [glg, glb, gw1, gb1, gw2, gb2]
        has = ctx.has
        ctx.st = None
        return (dtok, None, None, None, None, *[g if h else None for g, h in zip(grads, has)])


def _head_params(head) -> List[Optional[nn.Parameter]]:
    seq = head.output_head
    lns = [mm for mm in seq if isinstance(mm, nn.LayerNorm)]
    lins = [mm for mm in seq if isinstance(mm, nn.Linear)]
    ln_g, ln_b = (lns[0].weight, lns[0].bias) if lns else (None, None)
    w1, b1 = lins[0].weight, lins[0].bias
    w2, b2 = (lins[1].weight, lins[1].bias) if len(lins) > 1 else (None, None)
    return [ln_g, ln_b, w1, b1, w2, b2]


# ---------------------------------------------------------------------------
class _RawOutFn(torch.autograd.Function):
    """(x_raw_output [B, C, H, W], registers [B, R, C]) views of the final token buffer
    (model.py:147-148: return_raw_outputs); their gradients flow back into the token rows."""

    @staticmethod
    def forward(ctx, tok, geo):
        B, R, Hp, Wp, C = geo
        N = R + Hp * Wp
        xo = _empty((B, C, Hp, Wp), tok.dtype, tok.device)
        sp.rows_to_nchw(Rows(tok, C, Hp * Wp, N, R), xo)
        regs = _empty((B, R, C), tok.dtype, tok.device)
        if R:
            sp.copy_rows(tok, C, N * C, regs, C, R * C, B, R, C)
        ctx.geo, ctx.sdt = geo, tok.dtype
        return xo, regs

    @staticmethod
    def backward(ctx, dxo, dregs):
        B, R, Hp, Wp, C = ctx.geo
        N = R + Hp * Wp
        dtok = torch.zeros(B * N, C, dtype=ctx.sdt, device=(dxo if dxo is not None else dregs).device)
        if dxo is not None:
            sp.nchw_to_rows(dxo.contiguous(), Rows(dtok, C, Hp * Wp, N, R))
        if dregs is not None and R:
            sp.copy_rows(dregs.contiguous(), C, R * C, dtok, C, N * C, B, R, C)
        return dtok, None


# ---------------------------------------------------------------------------
# Sub-module forwards in training mode (Block(...)(x, reg), EncoderLayer, ConvMixer, the
# head, the LayerNorm / patcher / embedding leaves): the same per-sub-layer Functions on a
# token buffer built from (x NCHW, registers), with differentiable layout changes either side.
# ---------------------------------------------------------------------------
class _ToTokFn(torch.autograd.Function):
    """x [B, C, H, W] (may be None) + registers [B, R, C] (may be None) -> token rows
    [B*(R+HW), C] in dtype ``sdt`` (layers.py:271-275's flatten + concat)."""

    @staticmethod
    def forward(ctx, x, reg, sdt):
        if x is not None:
            B, C, H, W = x.shape
        else:
            (B, _, C), H, W = reg.shape, 0, 0
        R = 0 if reg is None else reg.shape[1]
        N = R + H * W
        dev = (x if x is not None else reg).device
        tok = _empty((B * N, C), sdt, dev)
        if x is not None:
            sp.nchw_to_rows(x.contiguous(), Rows(tok, C, H * W, N, R))
        if R:
            sp.copy_rows(reg.contiguous(), C, R * C, tok, C, N * C, B, R, C)
        ctx.geo = (B, R, H, W, C)
        ctx.dts = (None if x is None else x.dtype, None if reg is None else reg.dtype)
        return tok

    @staticmethod
    def backward(ctx, dtok):
        B, R, H, W, C = ctx.geo
        N = R + H * W
        dtok = dtok.contiguous()
        dx = None
        if ctx.dts[0] is not None:
            dx = _empty((B, C, H, W), ctx.dts[0], dtok.device)
            sp.rows_to_nchw(Rows(dtok, C, H * W, N, R), dx)
        dreg = None
        if ctx.dts[1] is not None:
            dreg = _empty((B, R, C), ctx.dts[1], dtok.device)
            if R:
                sp.copy_rows(dtok, C, N * C, dreg, C, R * C, B, R, C)
        return dx, dreg, None


def _enc_geo(e, B: int, N: int, mask):
    """(B, N) or (B, N, (bias, batch stride, head stride)): a mask takes the materialised attention
    (layers.py:289-298: SDPA attn_mask semantics for fast_att, masked_fill(mask == 0, -inf) for the
    manual path, via EncoderLayer._mask_bias as in eval)."""
    if mask is None:
        return (B, N)
    return (B, N, e._mask_bias(mask, B, N))


def train_conv_mixer(m, x: torch.Tensor) -> torch.Tensor:
    """ConvMixer.forward in train mode (layers.py:83-104): x [B, C, H, W] -> x."""
    dt = compute_dtype(x, m)
    B, C, H, W = x.shape
    tok = _ToTokFn.apply(x, None, stream_dtype(dt, C))
    tok = _MixerFn.apply(tok, (B, 0, H, W), m, dt, *_mixer_params(m))
    return _RawOutFn.apply(tok, (B, 0, H, W, C))[0]


def train_encoder(e, x: torch.Tensor, reg: torch.Tensor, mask=None):
    """EncoderLayer.forward in train mode (layers.py:268-316): (x, registers) -> (x, registers)."""
    dt = compute_dtype(x, e)
    B, C, H, W = x.shape
    tok = _ToTokFn.apply(x, reg, stream_dtype(dt, C))
    tok = _EncoderFn.apply(tok, _enc_geo(e, B, reg.shape[1] + H * W, mask), e, dt, _RNG(), *_enc_params(e))
    return _RawOutFn.apply(tok, (B, reg.shape[1], H, W, C))


def train_block(blk, x: torch.Tensor, reg: torch.Tensor, mask=None):
    """Block.forward in train mode (layers.py:381-386), one token buffer for the whole block."""
    dt = compute_dtype(x, blk)
    B, C, H, W = x.shape
    R = reg.shape[1]
    tok = _ToTokFn.apply(x, reg, stream_dtype(dt, C))
    rng = _RNG()

    def mixers(t):
        for mx in blk.conv_blocks:
            t = _MixerFn.apply(t, (B, R, H, W), mx, dt, *_mixer_params(mx))
        return t

    def enc(t):
        return _EncoderFn.apply(t, _enc_geo(blk.t_block, B, R + H * W, mask), blk.t_block, dt, rng,
                                *_enc_params(blk.t_block))

    tok = enc(mixers(tok)) if blk.conv_first else mixers(enc(tok))
    return _RawOutFn.apply(tok, (B, R, H, W, C))


def train_head(head, x: Optional[torch.Tensor], reg: Optional[torch.Tensor]) -> torch.Tensor:
    """ClassificationHead.forward in train mode (layers.py:447-465; dropout active): the
    register head reads only the registers, the pooling head only x."""
    if head.from_register:
        dt = compute_dtype(reg, head)
        B, R, C = reg.shape
        tok = _ToTokFn.apply(None, reg, stream_dtype(dt, C))
        return _HeadFn.apply(tok, (B, R, 0, R, C), head, dt, _RNG(), *_head_params(head))
    dt = compute_dtype(x, head)
    B, C, H, W = x.shape
    tok = _ToTokFn.apply(x, None, stream_dtype(dt, C))
    return _HeadFn.apply(tok, (B, 0, H * W, H * W, C), head, dt, _RNG(), *_head_params(head))


class _ChanLNFn(torch.autograd.Function):
    """Channel LayerNorm over dim 1 of NCHW (layers.py:12-24) with its backward; output in the
    promoted dtype of x and gamma (the reference's gamma * x + beta)."""

    @staticmethod
    def forward(ctx, x, g, b, eps):
        B, C, H, W = x.shape
        M = B * H * W
        odt = torch.promote_types(x.dtype, g.dtype)
        xr = _empty((M, C), odt, x.device)
        sp.nchw_to_rows(x.contiguous(), _dense(xr))
        a, st = _ln_fwd(_dense(xr), M, C, f32(g), f32(b), eps, odt)
        out = _empty((B, C, H, W), odt, x.device)
        sp.rows_to_nchw(_dense(a), out)
        ctx.st = (xr, st, f32(g), x.dtype, g.dtype, x.shape)
        return out

    @staticmethod
    def backward(ctx, dout):
        xr, st, g32, xdt, pdt, shp = ctx.st
        M, C = xr.shape
        dr = _empty((M, C), xr.dtype, xr.device)
        sp.nchw_to_rows(dout.contiguous(), _dense(dr))
        dxr = _empty((M, C), xr.dtype, xr.device)
        gg, gb = sp.ln_bwd(_dense(xr), st, g32, _dense(dr), _dense(dxr), M, C)
        dx = _empty(shp, xdt, xr.device)
        sp.rows_to_nchw(_dense(dxr), dx)
        ctx.st = None
        return dx, as_dtype(gg, pdt), as_dtype(gb, pdt), None


def train_layernorm(ln, x: torch.Tensor) -> torch.Tensor:
    compute_dtype(x, ln)  # device / dtype checks
    return _ChanLNFn.apply(x, ln.gamma, ln.beta, float(ln.eps))


class _PatchFn(torch.autograd.Function):
    """ConvPatcher (layers.py:28-42): stride-p convolution as patchify + GEMM; weight gradient
    dW = dY^T patches.  When the image requires grad (eager training), its gradient is the
    convolution's input gradient: dpatches = dY W on the GEMM, then sp.unpatchify (the adjoint of
    patchify); otherwise none is computed."""

    @staticmethod
    def forward(ctx, x, w, pat, dt):
        B, _, Hi, Wi = x.shape
        p = pat.patch_size
        Hp, Wp = Hi // p, Wi // p
        C = w.shape[0]
        kp = pat._kpad()
        patches = _empty((B * Hp * Wp, kp), dt, x.device)
        sp.patchify(x.contiguous(), patches, p, kp)
        wm = as_dtype(w.reshape(C, -1), dt)
        if kp != wm.shape[1]:
            wpad = torch.zeros(C, kp, dtype=dt, device=x.device)
            wpad[:, : wm.shape[1]].copy_(wm)
            wm = wpad
        rows = _linear(patches, wm, None, dt)
        out = _empty((B, C, Hp, Wp), dt, x.device)
        sp.rows_to_nchw(_dense(rows), out)
        need_dx = ctx.needs_input_grad[0]
        ctx.st = (patches, w.shape, 3 * p * p, dt, wm if need_dx else None, (x.shape, x.dtype), p, kp)
        return out

    @staticmethod
    def backward(ctx, dout):
        patches, wshape, k, dt, wm, (xshape, xdt), p, kp = ctx.st
        B, C, Hp, Wp = dout.shape
        dr = _empty((B * Hp * Wp, C), dt, dout.device)
        sp.nchw_to_rows(dout.contiguous(), _dense(dr))
        gw = _wgrad(dr, patches)[:, :k].contiguous().view(wshape)
        dx = None
        if wm is not None:  # input gradient: dpatches = dY . W (rows), then the adjoint of patchify
            dx = _empty(xshape, xdt, dout.device)
            sp.unpatchify(_dgrad(dr, wm), dx, p, kp)
        ctx.st = None
        return dx, gw, None, None


def train_patcher(pat, x: torch.Tensor) -> torch.Tensor:
    return _PatchFn.apply(x, pat.conv.weight, pat, compute_dtype(x, pat))


class _PosEmbFn(torch.autograd.Function):
    """EmbeddingLayer / ConvEmbedding in train mode (layers.py:152-168, :202-209): x [B, C, H, W]
    -> (act(x + pos), registers [B, R, C]) in x's dtype promoted with the tables' (x + an fp32
    table is fp32); gradients into x, the Eh / Ew tables or a trainable bone, and the register
    rows."""

    @staticmethod
    def forward(ctx, x, emb, nreg, eh, ew, bone, ereg):
        B, C, H, W = x.shape
        P = H * W
        dev = x.device
        odt = torch.promote_types(x.dtype, ereg.dtype)
        pos = emb._pos_table(H, W)  # fp32 [P, C]
        act = act_code(emb.activation)
        z = _empty((B * P, C), torch.float32, dev)
        sp.nchw_to_rows(x.contiguous(), _dense(z))
        sp.rowscale_add(_dense(z), _dense(z), B * P, C, resid=Rows(pos, C, P, 0, 0))
        y = z
        if act:
            y = _empty((B * P, C), torch.float32, dev)
            sp.rowscale_add(_dense(z), _dense(y), B * P, C, act=act)
        xo = _empty((B, C, H, W), odt, dev)
        sp.rows_to_nchw(_dense(y), xo)
        table, R = emb._register_rows(nreg)
        regs = _empty((B, R, C), odt, dev)
        if R:
            sp.copy_rows(table.contiguous(), C, 0, regs, C, R * C, B, R, C)
        ctx.st = dict(z=z if act else None, act=act, geo=(B, C, H, W, R), xdt=x.dtype, eh=eh, ew=ew, bone=bone,
                      k=getattr(emb, "kernel_size", 0), nreg_rows=ereg.shape[0], pdt=ereg.dtype)
        return xo, regs

    @staticmethod
    def backward(ctx, dxo, dregs):
        S = ctx.st
        B, C, H, W, R = S["geo"]
        P = H * W
        dev = (dxo if dxo is not None else dregs).device
        dz = torch.zeros((B * P, C), dtype=torch.float32, device=dev)
        if dxo is not None:
            sp.nchw_to_rows(dxo.contiguous(), _dense(dz))
        if S["act"]:
            sp.act_bwd(S["z"], dz, dz, B * P, C, S["act"])
        dx = None
        if ctx.needs_input_grad[0]:
            dx = _empty((B, C, H, W), S["xdt"], dev)
            sp.rows_to_nchw(_dense(dz), dx)
        dpos = _empty((P, C), torch.float32, dev)
        sp.seg_colsum(dz, dpos, P, B, 1, P, C)                              # sum over the batch
        geh = gew = gbone = None
        if S["eh"] is not None:
            geh = torch.zeros(S["eh"].shape, dtype=torch.float32, device=dev)
            gew = torch.zeros(S["ew"].shape, dtype=torch.float32, device=dev)
            sp.seg_colsum(dpos, geh, H, W, W, 1, C)                          # Eh indexed by h (rows)
            sp.seg_colsum(dpos, gew, W, H, 1, W, C)                          # Ew indexed by w (columns)
            geh, gew = as_dtype(geh, S["eh"].dtype), as_dtype(gew, S["ew"].dtype)
        elif S["bone"] is not None and ctx.needs_input_grad[5]:
            gbone = _empty(S["bone"].shape, torch.float32, dev)
            sp.avgpool_table_bwd(dpos, gbone, H, W, C, S["k"])
            gbone = as_dtype(gbone, S["bone"].dtype)
        greg = torch.zeros(S["nreg_rows"], C, dtype=torch.float32, device=dev)
        if R and dregs is not None:
            off = 1 if S["eh"] is None else 0  # ConvEmbedding takes Embedding rows 1..R (layers.py:206)
            sp.seg_colsum(dregs.contiguous(), greg[off:], R, B, 1, R, C)
        ctx.st = None
        return dx, None, None, geh, gew, gbone, as_dtype(greg, S["pdt"])


def train_pos_embedding(emb, x: torch.Tensor, num_registers: int):
    compute_dtype(x, emb)
    conv_emb = not hasattr(emb, "horizontal_embedding_layer")
    eh = None if conv_emb else emb.horizontal_embedding_layer.weight
    ew = None if conv_emb else emb.vertical_embedding_layer.weight
    bone = emb.bone if conv_emb and isinstance(emb.bone, nn.Parameter) else None
    return _PosEmbFn.apply(x, emb, num_registers, eh, ew, bone, emb.register_embedding_layer.weight)


def eval_forward(model, x: torch.Tensor, num_registers: int = 3, return_raw_outputs: bool = False):
    """MainModel.forward in eval mode along the training forward's kernels (model._fp32_stream_eval):
    the residual stream in fp32 as torch.autocast keeps it (training_tools.py:85), bf16 GEMM operands,
    dropout and drop path off (eval semantics, utility_layers.py:16-27), no autograd state kept."""
    global _NO_DROP
    prev = _NO_DROP
    _NO_DROP = True
    try:
        with torch.no_grad():
            return train_forward(model, x, num_registers, return_raw_outputs)
    finally:
        _NO_DROP = prev


def train_forward(model, x: torch.Tensor, num_registers: int = 3, return_raw_outputs: bool = False):
    """MainModel.forward in training mode (model.py:129-149 with dropout / drop path active)."""
    global _WPREP
    _WPREP = _prep_weights(model, compute_dtype(x, model))
    try:
        return _train_forward(model, x, num_registers, return_raw_outputs)
    finally:
        _WPREP = None


def _train_forward(model, x: torch.Tensor, num_registers: int, return_raw_outputs: bool):
    dt = compute_dtype(x, model)
    B, _, Hi, Wi = x.shape
    p = model.conv_init.patch_size
    Hp, Wp = Hi // p, Wi // p
    emb = model.embedding_layer
    conv_emb = not hasattr(emb, "horizontal_embedding_layer")
    if conv_emb:
        R = num_reg_rows(emb.register.shape[0], num_registers)
        eh = ew = None
    else:
        R = num_reg_rows(emb.max_num_registers, num_registers)
        eh, ew = emb.horizontal_embedding_layer.weight, emb.vertical_embedding_layer.weight
        if Hp > eh.shape[0] or Wp > ew.shape[0]:
            raise RuntimeError(f"image grid {Hp}x{Wp} exceeds max_image_size {[ew.shape[0], eh.shape[0]]}")
    N = R + Hp * Wp
    C = model.conv_init.conv.out_channels
    rng = _RNG()
    # the image goes in as is (patchify converts to the compute dtype), so a gradient reaches it
    tok = _EmbedFn.apply(x, (B, R, Hp, Wp, num_registers, stream_dtype(dt, C)), model, dt, model.conv_init.conv.weight, eh, ew,
                         emb.register_embedding_layer.weight)

    def enc(t, e):
        return _EncoderFn.apply(t, (B, N), e, dt, rng, *_enc_params(e))

    def mixers(t, blk):
        for mx in blk.conv_blocks:
            t = _MixerFn.apply(t, (B, R, Hp, Wp), mx, dt, *_mixer_params(mx))
        return t

    for blk in model.blocks:                                           # model.py:139-140, layers.py:381-386
        if blk.conv_first:
            tok = enc(mixers(tok, blk), blk.t_block)
        else:
            tok = mixers(enc(tok, blk.t_block), blk)
    tok = enc(tok, model.final_block.t_block)                          # model.py:143
    head = model.output_head
    logits = _HeadFn.apply(tok, (B, R, Hp * Wp, N, C), head, dt, rng, *_head_params(head))
    if not return_raw_outputs:
        return logits
    xo, regs = _RawOutFn.apply(tok, (B, R, Hp, Wp, C))
    return logits, xo, regs


# ---------------------------------------------------------------------------
# The same training forward / backward as an explicit tape (torch.compile path)
# ---------------------------------------------------------------------------
class _Ctx:
    """Stand-in for an autograd ctx: the Functions above keep their state in plain attributes."""


def tape_forward(model, x: torch.Tensor, num_registers: int, dt):
    """train_forward with every sub-layer Function's forward called directly and its ctx
    kept on a tape (no autograd graph), for the opaque torch.compile custom op
    (sdpnet_ops.train_forward).  Same kernels, same order, same RNG draws as train_forward,
    so a compiled step is bit-identical to an eager one."""
    global _WPREP
    _WPREP = _prep_weights(model, dt)
    try:
        return _tape_forward(model, x, num_registers, dt)
    finally:
        _WPREP = None


def _tape_forward(model, x: torch.Tensor, num_registers: int, dt):
    B, _, Hi, Wi = x.shape
    p = model.conv_init.patch_size
    Hp, Wp = Hi // p, Wi // p
    emb = model.embedding_layer
    conv_emb = not hasattr(emb, "horizontal_embedding_layer")
    if conv_emb:
        R = num_reg_rows(emb.register.shape[0], num_registers)
        eh = ew = None
    else:
        R = num_reg_rows(emb.max_num_registers, num_registers)
        eh, ew = emb.horizontal_embedding_layer.weight, emb.vertical_embedding_layer.weight
        if Hp > eh.shape[0] or Wp > ew.shape[0]:
            raise RuntimeError(f"image grid {Hp}x{Wp} exceeds max_image_size {[ew.shape[0], eh.shape[0]]}")
    N = R + Hp * Wp
    C = model.conv_init.conv.out_channels
    rng = _RNG()
    tape = []

    def run(fn, lead, params, *args):
        ctx = _Ctx()
        out = fn.forward(ctx, *args, *params)
        tape.append((fn, ctx, lead, params))
        return out

    xin = x if x.dtype == dt else as_dtype(x, dt)
    with torch.no_grad():
        tok = run(_EmbedFn, 4, [model.conv_init.conv.weight, eh, ew, emb.register_embedding_layer.weight],
                  xin, (B, R, Hp, Wp, num_registers, stream_dtype(dt, C)), model, dt)

        def enc(t, e):
            return run(_EncoderFn, 5, _enc_params(e), t, (B, N), e, dt, rng)

        def mixers(t, blk):
            for mx in blk.conv_blocks:
                t = run(_MixerFn, 4, _mixer_params(mx), t, (B, R, Hp, Wp), mx, dt)
            return t

        for blk in model.blocks:
            if blk.conv_first:
                tok = enc(mixers(tok, blk), blk.t_block)
            else:
                tok = mixers(enc(tok, blk.t_block), blk)
        tok = enc(tok, model.final_block.t_block)
        head = model.output_head
        logits = run(_HeadFn, 5, _head_params(head), tok, (B, R, Hp * Wp, N, C), head, dt, rng)
    return logits, tape


def tape_backward(tape, dlogits: torch.Tensor, params: List[torch.Tensor]) -> List[torch.Tensor]:
    """Replay the tape backwards; returns one fp32 gradient per entry of ``params`` (zeros for
    a parameter the forward did not use)."""
    grads = {}
    g = dlogits
    with torch.no_grad():
        for fn, ctx, lead, ps in reversed(tape):
            outs = fn.backward(ctx, g)
            g = outs[0]
            for prm, gp in zip(ps, outs[lead:]):
                if prm is not None and gp is not None:
                    grads[id(prm)] = gp if id(prm) not in grads else grads[id(prm)] + gp
    tape.clear()
    out = []
    for q in params:
        t = grads[id(q)].reshape(q.shape).to(q.dtype) if id(q) in grads else torch.zeros_like(q)
        if t._base is not None:  # e.g. the q/k/v slices of one fused dW: the op's outputs may not alias
            t = t.clone()
        out.append(t)
    return out


# ---------------------------------------------------------------------------
# Per-sub-layer form for torch.compile (sdpnet_ops.train_layer / train_layer_backward): one
# opaque op per patch-embedding / ConvMixer / EncoderLayer / head, each with its own autograd
# formula, so a compiled backward is a chain of per-layer ops and DDP's bucket hooks (and
# Dynamo's DDPOptimizer graph splits) see each layer's gradients as soon as its backward op
# returns -- the overlap the eager Functions give (training_tools.py:36-39 compiles DDP(model)).
# The forward session (seed source, prepared bf16 weights, geometry) lives on the model between
# the first and the last layer op of one forward; same Functions, same kernels, same RNG draws
# in the same order as train_forward, so the compiled step is bit-identical to the eager one.
# ---------------------------------------------------------------------------
def train_layers(model):
    """The sub-layers of a training forward in execution order: (kind, module)."""
    out = [("embed", model)]
    for blk in model.blocks:                                           # model.py:139-140
        mx = [("mixer", m) for m in blk.conv_blocks]
        en = [("enc", blk.t_block)]
        out += (mx + en) if blk.conv_first else (en + mx)
    out += [("enc", model.final_block.t_block), ("head", model.output_head)]
    return out


def layer_params(model, kind: str, mod) -> List[Optional[nn.Parameter]]:
    if kind == "embed":
        emb = model.embedding_layer
        conv_emb = not hasattr(emb, "horizontal_embedding_layer")
        eh = None if conv_emb else emb.horizontal_embedding_layer.weight
        ew = None if conv_emb else emb.vertical_embedding_layer.weight
        return [model.conv_init.conv.weight, eh, ew, emb.register_embedding_layer.weight]
    if kind == "mixer":
        return _mixer_params(mod)
    if kind == "enc":
        return _enc_params(mod)
    return _head_params(mod)


class _Session:
    pass


def layer_forward(model, layer: int, t: torch.Tensor, num_registers: int, dt, need_dx: bool = False):
    """Forward of sub-layer ``layer`` (train_layers order) with its ctx returned for the
    backward op.  Layer 0 takes the image and opens the session, the last layer closes it;
    need_dx: the image requires grad (layer 0 then keeps what its input gradient needs)."""
    global _WPREP
    kind, mod = train_layers(model)[layer]
    params = layer_params(model, kind, mod)
    ctx = _Ctx()
    ctx.needs_input_grad = (bool(need_dx),)
    if kind == "embed":
        S = _Session()
        B, _, Hi, Wi = t.shape
        p = model.conv_init.patch_size
        Hp, Wp = Hi // p, Wi // p
        emb = model.embedding_layer
        conv_emb = not hasattr(emb, "horizontal_embedding_layer")
        R = num_reg_rows(emb.register.shape[0] if conv_emb else emb.max_num_registers, num_registers)
        if not conv_emb:
            eh, ew = emb.horizontal_embedding_layer.weight, emb.vertical_embedding_layer.weight
            if Hp > eh.shape[0] or Wp > ew.shape[0]:
                raise RuntimeError(f"image grid {Hp}x{Wp} exceeds max_image_size {[ew.shape[0], eh.shape[0]]}")
        S.geo = (B, R, Hp, Wp, Hp * Wp + R, model.conv_init.conv.out_channels)
        S.dt = dt
        # _WPREP is valid only inside one layer op (cleared on every exit, as for the other layers);
        # the session keeps the prepared weights for the later layers, and a failed layer 0 leaves
        # no session behind
        try:
            _WPREP = _prep_weights(model, dt)
            S.wprep = _WPREP
            S.rng = _RNG()
            model._sdp_session = S
            C = S.geo[5]
            xin = t if t.dtype == dt else as_dtype(t, dt)
            with torch.no_grad():
                out = _EmbedFn.forward(ctx, xin, (B, R, Hp, Wp, num_registers, stream_dtype(dt, C)), model, dt,
                                       *params)
        except BaseException:
            model._sdp_session = None
            raise
        finally:
            _WPREP = None
        return out, (_EmbedFn, ctx, 4, params)
    S = getattr(model, "_sdp_session", None)
    if S is None:
        raise RuntimeError("sdpnet: training layer op run outside a forward (layer 0 opens it)")
    B, R, Hp, Wp, N, C = S.geo
    _WPREP = S.wprep
    try:
        with torch.no_grad():
            if kind == "mixer":
                out = _MixerFn.forward(ctx, t, (B, R, Hp, Wp), mod, S.dt, *params)
                rec = (_MixerFn, ctx, 4, params)
            elif kind == "enc":
                out = _EncoderFn.forward(ctx, t, (B, N), mod, S.dt, S.rng, *params)
                rec = (_EncoderFn, ctx, 5, params)
            else:
                out = _HeadFn.forward(ctx, t, (B, R, Hp * Wp, N, C), mod, S.dt, S.rng, *params)
                rec = (_HeadFn, ctx, 5, params)
    except BaseException:
        model._sdp_session = None  # an aborted forward closes the session (no stale weight copies)
        raise
    finally:
        _WPREP = None
    if kind == "head":
        model._sdp_session = None
    return out, rec


def layer_backward(rec, g: torch.Tensor):
    """(grad of the layer's input or None, one fp32 gradient per non-None parameter)."""
    fn, ctx, lead, params = rec
    with torch.no_grad():
        outs = fn.backward(ctx, g.contiguous())
    grads = []
    for prm, gp in zip(params, outs[lead:]):
        if prm is None:
            continue
        t = gp.reshape(prm.shape).to(prm.dtype) if gp is not None else torch.zeros_like(prm)
        if t._base is not None:  # e.g. the q/k/v slices of one fused dW: op outputs may not alias
            t = t.clone()
        grads.append(t)
    return outs[0], grads  # layer 0: the image gradient, or None when the image needs none


def raw_outputs(tok: torch.Tensor, geo):
    """(x_raw_output [B, C, H, W], registers [B, R, C]) of the final token buffer (model.py:147-148),
    _RawOutFn's forward without autograd (the compiled head-with-raw-outputs op)."""
    return _RawOutFn.forward(_Ctx(), tok, geo)


def add_raw_output_grads(dtok: torch.Tensor, dxo, dregs, geo) -> torch.Tensor:
    """dtok + the token-row gradient of the raw outputs (_RawOutFn.backward), summed by a HIP pass
    (the eager path leaves that sum to autograd's accumulation)."""
    if dxo is None and dregs is None:
        return dtok
    ctx = _Ctx()
    ctx.geo, ctx.sdt = geo, dtok.dtype
    draw, _ = _RawOutFn.backward(ctx, dxo, dregs)
    M, C = dtok.shape
    out = torch.empty_like(dtok)
    sp.rowscale_add(_dense(dtok), _dense(out), M, C, resid=_dense(draw))
    return out


def compiled_train_forward(model, x: torch.Tensor, num_registers: int, dtype_code: int,
                           return_raw_outputs: bool = False):
    """The training forward as a chain of sdpnet::train_layer ops (traced by Dynamo).  An image that
    requires grad gets its gradient from layer 0's backward op (the eager path's dY W + col2im);
    return_raw_outputs runs the head as sdpnet::train_head_raw, which also returns
    (x_raw_output, registers) and sums their gradients into the token rows in its backward op."""
    t = x
    B = x.shape[0]
    need_dx = int(x.requires_grad)
    layers = train_layers(model)
    for i, (kind, mod) in enumerate(layers):
        params = [q for q in layer_params(model, kind, mod) if q is not None]
        if return_raw_outputs and i == len(layers) - 1:
            p = model.conv_init.patch_size
            logits, xo, regs, _ = torch.ops.sdpnet.train_head_raw(t, params, model._sdp_handle, i, num_registers,
                                                                  dtype_code, B, x.shape[2] // p, x.shape[3] // p)
            return logits, xo, regs
        t, _ = torch.ops.sdpnet.train_layer(t, params, model._sdp_handle, i, num_registers, dtype_code, B,
                                            need_dx if i == 0 else 0)
    return t


# ---------------------------------------------------------------------------
# Loss and optimizer
# ---------------------------------------------------------------------------
class _CEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, eps, ignore_index=-100):
        loss = torch.zeros(1, dtype=torch.float32, device=logits.device)
        d = torch.empty_like(logits)
        if labels.is_floating_point():  # probability targets (CutMix / MixUp, dataset_generator.py:105-110)
            sp.ce_loss_soft(logits.contiguous(), labels.float().contiguous(), eps, 1.0, d, loss)
        else:
            sp.ce_loss(logits.contiguous(), labels, eps, 1.0, d, loss, ignore_index)
        ctx.save_for_backward(d)
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        (d,) = ctx.saved_tensors
        # g is the upstream scalar (the GradScaler scale, or 1): dlogits * g
        out = torch.empty_like(d)
        M, K = d.shape
        sc = g.float().reshape(1).expand(M).contiguous()
        sp.rowscale_add(_dense(d), _dense(out), M, K, scale=sc, sgrp=1)
        return out, None, None, None


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor, label_smoothing: float = 0.0,
                  ignore_index: int = -100) -> torch.Tensor:
    """nn.CrossEntropyLoss(label_smoothing=..., ignore_index=...)(logits, labels) as one HIP
    kernel (training_tools.py:76, :88).  ``labels`` are int64 class indices or float probability
    rows [B, K] (the CutMix / MixUp targets, dataset_generator.py:105-110).  As torch's 'mean'
    reduction: rows labelled ignore_index (default -100) are left out of the loss and of the
    divisor and get zero gradient; all rows ignored gives NaN.  Any other class index outside
    [0, K) gives a NaN loss (torch raises)."""
    return _CEFn.apply(logits, labels, float(label_smoothing), int(ignore_index))


# SDPNET_ADAMW_PTR_CACHE=0: upload the gradient address table every step with a blocking copy (A/B)
_GRAD_PTR_CACHE = os.environ.get("SDPNET_ADAMW_PTR_CACHE", "1") != "0"


class AdamW(torch.optim.Optimizer):
    """torch.optim.AdamW (training_tools.py:235; betas (0.9, 0.999), eps 1e-8, decoupled weight
    decay) as one multi-tensor HIP kernel, with torch.amp.GradScaler semantics folded in
    (training_tools.py:63-64, :91-99).

    ``step(grad_scale=S, max_norm=M)`` performs GradScaler.unscale_ (grads / S), the inf/nan
    check, clip_grad_norm_(M) and the AdamW update on device without a host sync.  A step
    whose gradients hold an inf/nan is skipped exactly as ``scaler.step(optimizer)`` skips
    ``optimizer.step()``: parameters, moments AND step counts stay as they were (the step
    counts live on the device, ``state[p]["step"]`` is a 0-d view of them).  ``grad_scale=None``
    unscales by the device scale ``self.scaler[0]``; multiply the loss by the same value with
    ``opt.scale(loss)`` and a backoff takes effect on the next step without any host sync.
    The scale updates like torch.amp.GradScaler (growth 2, backoff 0.5, interval 2000) unless
    ``update_scaler=False``.  Parameters whose ``grad`` is None are left out of the step
    (no decay, no moment update, no step count), as torch does.  The device work lists are
    rebuilt whenever a parameter, its state tensors or the set of parameters with gradients
    change (``load_state_dict``, ``add_param_group``, a reallocated tensor)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, init_scale=65536.0,
                 growth_interval=2000):
        self._tables = None
        self._sig = None
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.growth_interval = growth_interval
        self._init_scale = float(init_scale)
        self.scaler = None
        self.state_buf = None

    def add_param_group(self, param_group):
        super().add_param_group(param_group)
        self._tables = None

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._tables = None

    def _ensure_device_state(self, dev):
        if self.scaler is None:
            self.state_buf = torch.zeros(2, dtype=torch.float32, device=dev)
            self.scaler = torch.tensor([self._init_scale, 0.0], dtype=torch.float32, device=dev)
            self.scaler[1:].view(torch.int32).zero_()

    def scale(self, loss: torch.Tensor) -> torch.Tensor:
        """GradScaler.scale(loss): loss * the device scale (no host sync)."""
        self._ensure_device_state(loss.device)
        return loss * self.scaler[0]

    def _signature(self):
        sig = []
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    sig.append(None)
                    continue
                st = self.state.get(p)
                if not st:
                    sig.append(-1)
                    continue
                sig.append((p.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(), id(st["step"])))
        return sig

    def _build(self, dev):
        bb = sp.lib().sdp_mt_block_bytes()
        self._tables = []
        groups = [[p for p in group["params"] if p.grad is not None] for group in self.param_groups]
        counts = []
        for ps in groups:
            for p in ps:
                if p.dtype != torch.float32 or not p.is_contiguous() or p.device != dev:
                    raise TypeError("sdpnet AdamW: fp32 contiguous parameters on one device only")
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                for k in ("exp_avg", "exp_avg_sq"):  # e.g. a state dict loaded to another device
                    t = st[k]
                    if t.device != dev or t.dtype != torch.float32 or not t.is_contiguous():
                        st[k] = t.to(device=dev, dtype=torch.float32).contiguous()
                counts.append(float(st["step"]))
        # one device array of step counts for every table (sdp_adamw_finish advances it in one launch)
        self._steps = torch.tensor(counts, dtype=torch.float32, device=dev)
        base = 0
        for ps in groups:
            steps = self._steps[base:base + len(ps)]
            for i, p in enumerate(ps):
                self.state[p]["step"] = steps[i]
            base += len(ps)
            blocks = []
            for ti, p in enumerate(ps):
                for s0 in range(0, p.numel(), 4096):
                    blocks.append((ti, s0))
            raw = bytearray(bb * len(blocks))
            for i, (t, s0) in enumerate(blocks):
                struct.pack_into("<iiq", raw, i * bb, t, 0, s0)
            btab = (torch.frombuffer(raw, dtype=torch.uint8).to(dev) if blocks
                    else torch.empty(0, dtype=torch.uint8, device=dev))
            sizes = torch.tensor([p.numel() for p in ps], dtype=torch.int64, device=dev)

            def ptrs(ts):
                return torch.tensor([t.data_ptr() for t in ts], dtype=torch.int64, device=dev)
            self._tables.append(dict(params=ps, blocks=btab, nblocks=len(blocks), sizes=sizes, pp=ptrs(ps),
                                     m1=ptrs([self.state[p]["exp_avg"] for p in ps]),
                                     m2=ptrs([self.state[p]["exp_avg_sq"] for p in ps]), steps=steps))
        nb = sum(t["nblocks"] for t in self._tables)
        self._partials = torch.zeros(max(1, nb), dtype=torch.float32, device=dev)
        self._ensure_device_state(dev)
        self._sig = self._signature()

    def _grad_ptrs(self, tab, dev) -> torch.Tensor:
        """Device array of the table's gradient addresses.  Uploaded only when they change (set_to_none
        gradients usually come back at the same addresses), from pinned memory without blocking: a
        pageable torch.tensor(..., device=) waits for the whole queued backward, so the GPU idled while
        the host prepared the optimizer and the next step (~2 ms per XL step)."""
        ptrs = [p.grad.data_ptr() for p in tab["params"]]
        if _GRAD_PTR_CACHE and tab.get("gptrs") == ptrs:
            return tab["g"]
        h = torch.tensor(ptrs, dtype=torch.int64)
        if _GRAD_PTR_CACHE:
            h = h.pin_memory()
        tab["g"] = h.to(dev, non_blocking=_GRAD_PTR_CACHE)
        tab["gptrs"] = ptrs
        return tab["g"]

    @torch.no_grad()
    def step(self, closure=None, grad_scale: Optional[float] = 1.0, max_norm: float = 0.0,
             update_scaler: bool = True):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        dev = None
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is not None:
                    dev = p.device
                    break
            if dev is not None:
                break
        if dev is None:
            return loss
        self._ensure_device_state(dev)
        if self._tables is None or self._signature() != self._sig:
            self._build(dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        L = sp.lib()
        gptr = []
        off = 0
        for tab in self._tables:  # per-block sums of squares, then one fixed-order sum (bit-reproducible)
            g = self._grad_ptrs(tab, dev)
            gptr.append(g)
            sp._check(L.sdp_grad_sumsq_parts(g.data_ptr(), tab["sizes"].data_ptr(), tab["blocks"].data_ptr(),
                                             tab["nblocks"], self._partials.data_ptr() + 4 * off,
                                             self.state_buf.data_ptr(), stream), "grad_sumsq")
            off += tab["nblocks"]
        sp._check(L.sdp_sum_partials(self._partials.data_ptr(), off, self.state_buf.data_ptr(), stream),
                  "sum_partials")
        dscale = self.scaler.data_ptr() if grad_scale is None else None
        inv = 1.0 if grad_scale is None else 1.0 / float(grad_scale)
        for tab, g, group in zip(self._tables, gptr, self.param_groups):
            if not tab["params"]:
                continue
            b1, b2 = group["betas"]
            sp._check(L.sdp_adamw_dev(tab["pp"].data_ptr(), g.data_ptr(), tab["m1"].data_ptr(),
                                      tab["m2"].data_ptr(), tab["sizes"].data_ptr(), tab["blocks"].data_ptr(),
                                      tab["nblocks"], self.state_buf.data_ptr(), float(group["lr"]), float(b1),
                                      float(b2), float(group["eps"]), float(group["weight_decay"]),
                                      tab["steps"].data_ptr(), dscale, inv, float(max_norm), stream), "adamw")
        # step counts advance only if the step was taken; scale update; state reset
        sp._check(L.sdp_adamw_finish(self.state_buf.data_ptr(), self.scaler.data_ptr() if update_scaler else None,
                                     2.0, 0.5, self.growth_interval, self._steps.data_ptr(), self._steps.numel(),
                                     stream), "adamw_finish")
        return loss
