"""ctypes binding of libsdpnet_hip.so (include/sdpnet_hip.h) + thin tensor wrappers.

This is the only place Python touches the C ABI.  Every wrapper:
  * checks device / dtype / contiguity / shape on the host,
  * passes raw device pointers and sizes (no torch types cross the boundary),
  * launches on the caller's current HIP stream (torch.cuda.current_stream()),
  * raises RuntimeError naming the op if the library returns a non-zero code.

There is no fallback: if the shared library is missing or cannot be loaded,
``lib()`` raises, and every op that needs it raises with it.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional, Tuple

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SDPNET_HIP_LIB", os.path.join(_HERE, "lib", "libsdpnet_hip.so"))

F32, BF16 = 0, 1
ACT_CODES = {"none": 0, "gelu": 1, "relu": 2, "tanh": 3, "sigmoid": 4, "leaky_relu": 5, "selu": 6, "kelu": 7}

_i32, _i64, _f32, _vp, _u64 = ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p, ctypes.c_uint64
_HIP_NOT_SUPPORTED = 801  # hipErrorNotSupported
_ROWMAP = [_i32, _i64, _i32]

# Signatures, in the order of include/sdpnet_hip.h.
_SIGS = {
    "sdp_version": ([], ctypes.c_char_p),
    "sdp_gemm": ([_i32, _vp, _i64, *_ROWMAP, _vp, _i64, _vp, _vp, _i64, *_ROWMAP, _vp, _i64, *_ROWMAP,
                  _i32, _i32, _i32, _i32, _i32, _vp], _i32),
    "sdp_gemm_ln": ([_i32, _vp, _i64, *_ROWMAP, _vp, _i64, _vp, _vp, _i64, *_ROWMAP, _vp, _i64, *_ROWMAP,
                     _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp], _i32),
    "sdp_gemm_variant": ([_i32, _i32, _i32, _i32], _i32),
    "sdp_gemm_force_generic": ([_i32], _i32),
    "sdp_gemm_set_fast_kernel": ([_i32], _i32),
    "sdp_gemm_set_store_policy": ([_i32], _i32),
    "sdp_gemm_set_epi_spec": ([_i32], _i32),
    "sdp_gemm_set_kloop_phases": ([_i32], _i32),
    "sdp_gemm_set_ct": ([_i32, _i32, _i32, _i32], _i32),
    "sdp_gemm_set_timeline": ([_vp, _i32], _i32),
    "sdp_gemm_timeline_count": ([], _i32),
    "sdp_debug_skip": ([_i32], _i32),
    "sdp_build_info": ([], _i32),
    "sdp_gemm_set_group_m": ([_i32], _i32),
    "sdp_gemm_set_exact_gelu": ([_i32], _i32),
    "sdp_mt_cast_transpose_entry_bytes": ([], _i32),
    "sdp_mt_cast_transpose": ([_vp, _vp, _i32, _vp], _i32),
    "sdp_gemm_wgrad": ([_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i32, _i32, _i32, _i32, _vp, _vp], _i32),
    "sdp_layernorm": ([_i32, _vp, _i64, *_ROWMAP, _vp, _vp, _f32, _vp, _i64, *_ROWMAP, _i32, _i32, _vp], _i32),
    "sdp_qk_headnorm": ([_i32, _vp, _i64, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _f32, _vp], _i32),
    "sdp_rowstats": ([_i32, _vp, _i64, *_ROWMAP, _f32, _vp, _i32, _i32, _vp], _i32),
    "sdp_row_partials": ([_i32, _vp, _i64, *_ROWMAP, _i32, _i32, _vp, _vp], _i32),
    "sdp_ln_stats": ([_vp, *_ROWMAP, _i32, _i32, _f32, _vp, _vp], _i32),
    "sdp_dwconv": ([_i32, _vp, _i64, *_ROWMAP, _vp, _vp, _vp, _vp, _vp, _vp, _i64, *_ROWMAP, _i32, _i32, _i32,
                    _i32, _i32, _vp], _i32),
    "sdp_dwconv_set_kernel": ([_i32], _i32),
    "sdp_attention": ([_i32, _vp, _i64, _vp, _i64, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _f32, _vp, _i64,
                       _i64, _vp], _i32),
    "sdp_attention_variant": ([_i32, _i32, _i32, _i32, _i32], _i32),
    "sdp_attention_set_kernel": ([_i32], _i32),
    "sdp_patchify": ([_i32, _vp, _i32, _vp, _i32, _i32, _i32, _i32, _i32, _vp], _i32),
    "sdp_unpatchify": ([_i32, _vp, _i32, _vp, _i32, _i32, _i32, _i32, _i32, _vp], _i32),
    "sdp_pos_table": ([_vp, _vp, _vp, _i32, _i32, _i32, _vp], _i32),
    "sdp_avgpool_table_bwd": ([_vp, _i32, _i32, _i32, _i32, _vp, _i32, _i32, _vp], _i32),
    "sdp_avgpool_table": ([_vp, _i32, _i32, _vp, _i32, _i32, _i32, _i32, _vp], _i32),
    "sdp_copy_rows": ([_i32, _vp, _i64, _i64, _i32, _vp, _i64, _i64, _i32, _i32, _i32, _vp], _i32),
    "sdp_nchw_add_table": ([_i32, _vp, _vp, _i32, _i32, _i32, _vp], _i32),
    "sdp_act": ([_i32, _vp, _vp, _i64, _i32, _vp], _i32),
    "sdp_group_mean": ([_i32, _vp, _i64, *_ROWMAP, _i32, _vp, _i64, _i32, _i32, _i32, _vp], _i32),
    "sdp_nchw_to_rows": ([_i32, _vp, _i32, _vp, _i64, *_ROWMAP, _i32, _i32, _i32, _vp], _i32),
    "sdp_rows_to_nchw": ([_i32, _vp, _i64, *_ROWMAP, _i32, _vp, _i32, _i32, _i32, _vp], _i32),
    "sdp_cast": ([_i32, _vp, _i32, _vp, _i64, _vp], _i32),
    "sdp_fold_ln_weight": ([_vp, _vp, _vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp, _vp], _i32),
    "sdp_val_preprocess": ([_vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp,
                            _vp, _vp, _i64, _i32, _i32, _vp, _vp, _vp], _i32),
    "sdp_logits_metrics": ([_i32, _vp, _i64, _vp, _i32, _i32, _f32, _vp, _vp], _i32),
    # training step (train.hip)
    "sdp_gemm_flex": ([_i32, _i32, _i32, _i32, _vp, _i64, _i64, _i64, _vp, _i64, _i64, _i64, _vp, _i64, _i64, _i64,
                       _i32, _i32, _i32, _i32, _i32, _i32, _i64, _f32, _i32, _vp], _i32),
    "sdp_transpose": ([_i32, _vp, _i64, _vp, _i64, _i32, _i32, _vp], _i32),
    "sdp_seg_colsum": ([_i32, _vp, _i64, _i32, _i32, _i64, _i64, _i32, _vp, _i64, _f32, _i32, _vp], _i32),
    "sdp_act_fwd": ([_i32, _vp, _i64, _vp, _i64, _i32, _i32, _i32, _f32, _u64, _vp], _i32),
    "sdp_act_bwd": ([_i32, _vp, _i64, _vp, _i64, _vp, _i64, _i32, _i32, _i32, _f32, _u64, _vp], _i32),
    "sdp_rowscale_add": ([_i32, _vp, _i64, *_ROWMAP, _vp, _i32, _vp, _i64, *_ROWMAP, _vp, _i64, *_ROWMAP, _i32, _i32,
                          _vp], _i32),
    "sdp_act_rowscale_add": ([_i32, _i32, _vp, _i64, *_ROWMAP, _vp, _i32, _vp, _i64, *_ROWMAP, _vp, _i64, *_ROWMAP, _i32, _i32,
                          _vp], _i32),
    "sdp_attn_set_per_cu": ([_i32], _i32),
    "sdp_gemm_train_epi": ([_i32, _vp, _i64, _vp, _i64, _vp, _vp, _i64, _vp, _i64, _vp, _i64, _i32, _i32, _i32,
                            _i32, _f32, _u64, _vp], _i32),
    "sdp_rowscale_add_mixed": ([_i32, _i32, _i32, _vp, _i64, *_ROWMAP, _vp, _i32, _vp, _i64, *_ROWMAP, _vp, _i64,
                                *_ROWMAP, _i32, _i32, _vp], _i32),
    "sdp_rowscale_add_dropout": ([_i32, _i32, _vp, _i64, *_ROWMAP, _vp, _i32, _vp, _i64, *_ROWMAP, _vp, _i64,
                                  *_ROWMAP, _i32, _i32, _f32, _u64, _i32, _vp], _i32),
    "sdp_ln_fwd_mixed": ([_i32, _i32, _vp, _i64, *_ROWMAP, _f32, _vp, _vp, _vp, _vp, _i64, *_ROWMAP, _i32, _i32, _vp],
                         _i32),
    "sdp_add_ln_fwd": ([_i32, _i32, _i32, _i32, _vp, _i64, *_ROWMAP, _vp, _i32, _vp, _i64, *_ROWMAP, _vp, _i64, *_ROWMAP,
                        _f32, _u64, _i32, _f32, _vp, _vp, _vp, _vp, _i64, *_ROWMAP, _i32, _i32, _vp, _vp, _vp, _i32,
                        _i32, _i32, _vp], _i32),
    "sdp_ln_bwd_mixed": ([_i32, _i32, _vp, _i64, *_ROWMAP, _vp, _vp, _vp, _i64, *_ROWMAP, _vp, _i64, *_ROWMAP, _vp,
                          _i64, *_ROWMAP, _i32, _i32, _vp, _vp], _i32),
    "sdp_ln_bwd_fused": ([_i32, _i32, _vp, _i64, *_ROWMAP, _vp, _vp, _vp, _i64, *_ROWMAP, _vp, _i64, *_ROWMAP, _vp,
                          _i64, *_ROWMAP, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _i64, _i32, _f32, _u64, _i32,
                          _vp, _i64, _vp, _vp, _i32, _i32, _i32, _vp], _i32),
    "sdp_ln_apply": ([_i32, _vp, _i64, *_ROWMAP, _vp, _vp, _vp, _vp, _i64, *_ROWMAP, _i32, _i32, _vp], _i32),
    "sdp_ln_bwd_blocks": ([_i32], _i32),
    "sdp_ln_fwd": ([_i32, _vp, _i64, *_ROWMAP, _f32, _vp, _vp, _vp, _vp, _i64, *_ROWMAP, _i32, _i32, _vp], _i32),
    "sdp_ln_bwd": ([_i32, _vp, _i64, *_ROWMAP, _vp, _vp, _vp, _i64, *_ROWMAP, _vp, _i64, *_ROWMAP, _vp, _i64,
                    *_ROWMAP, _i32, _i32, _vp, _vp], _i32),
    "sdp_softmax_fwd": ([_i32, _vp, _i64, _vp, _vp, _i64, _i32, _i32, _i32, _f32, _f32, _u64, _vp], _i32),
    "sdp_softmax_fwd_mask": ([_i32, _vp, _i64, _vp, _vp, _i64, _i32, _i32, _i32, _f32, _f32, _u64, _vp, _i64, _i64,
                              _i32, _vp], _i32),
    "sdp_softmax_bwd": ([_i32, _vp, _i64, _vp, _i64, _vp, _i64, _i32, _i32, _i32, _f32, _u64, _vp], _i32),
    "sdp_dw_wgrad_chunks": ([_i32], _i32),
    "sdp_dw_wgrad": ([_i32, _vp, _i64, *_ROWMAP, _vp, _i64, *_ROWMAP, _i32, _i32, _i32, _i32, _i32, _vp, _vp], _i32),
    "sdp_ce_loss": ([_i32, _vp, _i64, _vp, _i32, _i32, _f32, _f32, _vp, _i64, _vp, _vp], _i32),
    "sdp_ce_loss_ignore": ([_i32, _vp, _i64, _vp, _i32, _i32, _f32, _f32, _i64, _vp, _i64, _vp, _vp], _i32),
    "sdp_ce_count": ([_vp, _i32, _i64, _vp, _vp], _i32),
    "sdp_ce_loss_counted": ([_i32, _vp, _i64, _vp, _i32, _i32, _f32, _f32, _i64, _vp, _vp, _i64, _vp, _vp], _i32),
    "sdp_ce_loss_soft": ([_i32, _vp, _i64, _vp, _i64, _i32, _i32, _f32, _f32, _vp, _i64, _vp, _vp], _i32),
    "sdp_mt_block_bytes": ([], _i32),
    "sdp_grad_sumsq": ([_vp, _vp, _vp, _i32, _vp, _vp], _i32),
    "sdp_adamw": ([_vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _f32, _f32, _f32, _f32, _f32, _i32, _f32, _f32, _vp], _i32),
    "sdp_scaler_update": ([_vp, _vp, _f32, _f32, _i32, _vp], _i32),
    "sdp_adamw_dev": ([_vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _f32, _f32, _f32, _f32, _f32, _vp, _vp, _f32, _f32,
                       _vp], _i32),
    "sdp_adamw_finish": ([_vp, _vp, _f32, _f32, _i32, _vp, _i32, _vp], _i32),
    "sdp_grad_sumsq_parts": ([_vp, _vp, _vp, _i32, _vp, _vp, _vp], _i32),
    "sdp_sum_partials": ([_vp, _i32, _vp, _vp], _i32),
    "sdp_attn_train_applies": ([_i32, _i32, _i32], _i32),
    "sdp_attn_train_fwd": ([_i32, _vp, _i64, _vp, _i64, _vp, _i32, _i32, _i32, _i32, _f32, _f32, _u64, _vp], _i32),
    "sdp_attn_train_bwd": ([_i32, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _i64, _i32,
                            _i32, _i32, _i32, _f32, _f32, _u64, _vp], _i32),
    "sdp_attn_dropout_mask": ([_vp, _i32, _i32, _f32, _u64, _vp], _i32),
}

_lib = None

# Fast-GEMM launch timeline (bench.py's roofline): while active, every launch that takes the
# 8-phase kernel writes its {first workgroup start, last workgroup end} (s_memrealtime ticks,
# 100 MHz) into one slot of a device buffer -- also inside a captured and replayed graph, where
# HIP events cannot be recorded -- and the host side records (slot, M, N, K, flops, bytes).
_TL = None
TIMELINE_TICK_NS = 10.0


def gemm_timeline_begin(buf: torch.Tensor):
    """Start recording fast-GEMM launches into buf (int64 device tensor, 2 entries per slot)."""
    global _TL
    _req(buf.is_cuda and buf.dtype == torch.int64 and buf.is_contiguous() and buf.numel() >= 2)
    lib().sdp_gemm_set_timeline(buf.data_ptr(), buf.numel() // 2)
    _TL = []


def gemm_timeline_end():
    """Stop recording; returns [(slot, M, N, K, flops, algorithmic_bytes)] in launch order."""
    global _TL
    lib().sdp_gemm_set_timeline(None, 0)
    out, _TL = _TL, None
    return out or []


def lib():
    """Load libsdpnet_hip.so (after torch, so it binds torch's HIP runtime)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"sdpnet: HIP extension not built: {LIB_PATH} is missing "
                               "(run `python -c 'import __graft_entry__ as g; g.build()'` or `make -C sdp-net_amd/csrc`)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        # A/B switches of the benchmarks (bench.py records every SDPNET_* variable).  A selection the
        # loaded library does not offer (the 4-phase k-loop, the run-time-flag epilogue, the NT-store
        # policy and attention tiers 2 / 6 exist only in the diagnostic build) raises instead of
        # silently running the default.
        def knob(var, setter, what):
            v = os.environ.get(var)
            if v and setter(int(v)) < 0:
                raise RuntimeError(f"{var}={v}: {what} not available in {LIB_PATH} (sdp_build_info() = "
                                   f"{L.sdp_build_info()}); the A/B arms of earlier rounds are compiled only "
                                   "into the diagnostic library (make -C sdp-net_amd/csrc stamps)")
        knob("SDPNET_GEMM_KERNEL", L.sdp_gemm_set_fast_kernel, "bf16 fast GEMM kernel id")
        knob("SDPNET_GEMM_NT_STORE", L.sdp_gemm_set_store_policy, "GEMM store policy")
        knob("SDPNET_GEMM_EPI_SPEC", L.sdp_gemm_set_epi_spec, "GEMM epilogue specialisation")
        knob("SDPNET_GEMM_KLOOP_PHASES", L.sdp_gemm_set_kloop_phases, "GEMM k-loop phases")
        v = os.environ.get("SDPNET_GEMM_CT")  # cross-tile GEMM: "tiles[,re[,kmax[,nmax]]]"
        if v:
            a = [int(u) for u in v.split(",")] + [2, 1024, 1 << 30][len(v.split(",")) - 1:]
            if L.sdp_gemm_set_ct(a[0], a[1], a[2], a[3]) < -1:
                raise RuntimeError(f"SDPNET_GEMM_CT={v}: invalid cross-tile setting")
        kern = os.environ.get("SDPNET_DEBUG_SKIP")  # timing experiments, diagnostic library only
        if kern and int(kern) and L.sdp_debug_skip(int(kern)) < 0:
            raise RuntimeError("SDPNET_DEBUG_SKIP needs the diagnostic library (make -C sdp-net_amd/csrc stamps, "
                               "SDPNET_HIP_LIB=sdp-net_amd/lib_stamps/libsdpnet_hip.so); the product library "
                               "has no kernel-skip paths")
        kern = os.environ.get("SDPNET_GEMM_GROUP_M")  # tile raster of the 8-phase GEMM (-1 auto, 1 row-major)
        if kern:
            L.sdp_gemm_set_group_m(int(kern))
        knob("SDPNET_DW_KERNEL", L.sdp_dwconv_set_kernel, "depthwise-conv tier")
        knob("SDPNET_ATTN_KERNEL", L.sdp_attention_set_kernel, "attention tier")
        kern = os.environ.get("SDPNET_ATTN_PER_CU")  # fa4 workgroups per CU (0 = occupancy-derived)
        if kern:
            L.sdp_attn_set_per_cu(int(kern))
        _lib = L
    return _lib


def exported_symbols():
    return list(_SIGS.keys())


def _req(cond, what: str = "argument check"):
    """Boundary validation that survives ``python -O`` (unlike assert)."""
    if not cond:
        raise ValueError(f"sdpnet HIP op: invalid arguments ({what})")


def _check(rc: int, name: str):
    if rc != 0:
        raise RuntimeError(f"sdpnet HIP op {name} failed with hip error code {rc}")


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def dcode(dtype: torch.dtype) -> int:
    if dtype == torch.float32:
        return F32
    if dtype == torch.bfloat16:
        return BF16
    raise TypeError(f"sdpnet HIP path supports float32 and bfloat16, got {dtype}")


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _need_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("sdpnet HIP op called with a CPU tensor; the HIP path has no CPU fallback")


@dataclass
class Rows:
    """A row-addressed operand: logical row m -> physical row
    (m // grp) * gstride + off + m % grp of ``t`` (row stride ``ld`` elements).
    grp <= 0: dense."""
    t: torch.Tensor
    ld: int
    grp: int = 0
    gstride: int = 0
    off: int = 0

    def args(self):
        return [self.t.data_ptr(), self.ld, self.grp, self.gstride, self.off]

    def map(self):
        return [self.grp, self.gstride, self.off]


def dense(t: torch.Tensor) -> Rows:
    _req(t.is_contiguous())
    return Rows(t, t.shape[-1])


# ---------------------------------------------------------------------------
def gemm(x: Rows, w: torch.Tensor, y: Rows, M: int, N: int, K: int, bias: Optional[torch.Tensor] = None,
         resid: Optional[Rows] = None, act: int = 0, resid_pre: bool = False,
         ln: Optional[Tuple[torch.Tensor, torch.Tensor]] = None, part: Optional[torch.Tensor] = None):
    """y = epilogue(x . w^T).  ln = (stats [M,2] (mean, rstd) per logical row of x,
    colsum [N] of the LN-folded weight): LayerNorm folded into the GEMM
    (w = W * gamma, bias = beta . W^T + b).  part: token-row partial statistics
    buffer [rows, ceil(N/64), 2] the output rows' {mean, M2} are written to."""
    _need_cuda(x.t, w, y.t, bias)
    dt = dcode(x.t.dtype)
    _req(w.dtype == x.t.dtype == y.t.dtype and w.is_contiguous() and w.shape[0] >= N)
    _req(bias is None or (bias.dtype == torch.float32 and bias.is_contiguous()))
    if resid is not None:
        _req(resid.t.dtype == x.t.dtype)
        r = [resid.t.data_ptr(), resid.ld, *resid.map()]
    else:
        r = [None, 0, 0, 0, 0]
    tl = _TL
    if tl is not None:
        slot0 = lib().sdp_gemm_timeline_count()
    if ln is None and part is None:
        rc = lib().sdp_gemm(dt, *x.args(), w.data_ptr(), w.stride(0), _ptr(bias), *r, *y.args(), M, N, K, act,
                            int(bool(resid_pre)), _stream(y.t))
    else:
        if ln is not None:
            _req(ln[0].dtype == ln[1].dtype == torch.float32 and ln[0].numel() >= 2 * M and ln[1].numel() >= N)
        _req(part is None or part.dtype == torch.float32)
        rc = lib().sdp_gemm_ln(dt, *x.args(), w.data_ptr(), w.stride(0), _ptr(bias), *r, *y.args(), M, N, K, act,
                               int(bool(resid_pre)), _ptr(ln[0]) if ln else None, _ptr(ln[1]) if ln else None,
                               _ptr(part), _stream(y.t))
    _check(rc, "gemm")
    if tl is not None and lib().sdp_gemm_timeline_count() > slot0:
        es = x.t.element_size()
        nbytes = es * (M * K + N * K + M * N * (2 if resid is not None else 1)) + (4 * N if bias is not None else 0)
        tl.append((slot0, M, N, K, 2.0 * M * N * K, nbytes))


def layernorm(x: Rows, gamma: torch.Tensor, beta: torch.Tensor, eps: float, y: Rows, M: int, C: int):
    _need_cuda(x.t, y.t, gamma, beta)
    dt = dcode(x.t.dtype)
    _req(y.t.dtype == x.t.dtype and gamma.dtype == beta.dtype == torch.float32)
    rc = lib().sdp_layernorm(dt, *x.args(), gamma.data_ptr(), beta.data_ptr(), float(eps), *y.args(), M, C,
                             _stream(y.t))
    _check(rc, "layernorm")


def qk_headnorm(qkv: torch.Tensor, rows: int, n_head: int, head_dim: int, gq, bq, gk, bk, eps: float = 1e-5):
    _need_cuda(qkv, gq, bq, gk, bk)
    rc = lib().sdp_qk_headnorm(dcode(qkv.dtype), qkv.data_ptr(), qkv.stride(0), rows, n_head, head_dim,
                               gq.data_ptr(), bq.data_ptr(), gk.data_ptr(), bk.data_ptr(), float(eps), _stream(qkv))
    _check(rc, "qk_headnorm")


def row_partials(x: Rows, M: int, C: int, part: torch.Tensor):
    """part[phys_row] = per-64-column {mean, M2} of the rows of x (LN statistics by parts)."""
    _need_cuda(x.t, part)
    _req(part.dtype == torch.float32)
    rc = lib().sdp_row_partials(dcode(x.t.dtype), *x.args(), M, C, part.data_ptr(), _stream(part))
    _check(rc, "row_partials")


def ln_stats(part: torch.Tensor, rows: Rows, M: int, C: int, eps: float, stats: torch.Tensor):
    """stats[m] = (mean, rstd) of logical row m of ``rows`` (its map over ``part``'s physical rows)."""
    _need_cuda(part, stats)
    _req(part.dtype == stats.dtype == torch.float32 and stats.numel() >= 2 * M)
    rc = lib().sdp_ln_stats(part.data_ptr(), *rows.map(), M, C, float(eps), stats.data_ptr(), _stream(stats))
    _check(rc, "ln_stats")


def rowstats(x: Rows, eps: float, stats: torch.Tensor, M: int, C: int):
    _need_cuda(x.t, stats)
    _req(stats.dtype == torch.float32 and stats.numel() >= 2 * M)
    rc = lib().sdp_rowstats(dcode(x.t.dtype), *x.args(), float(eps), stats.data_ptr(), M, C, _stream(stats))
    _check(rc, "rowstats")


def dwconv(x: Rows, weight: torch.Tensor, bias: Optional[torch.Tensor], y: Rows, B: int, H: int, W: int, C: int,
           k: int, stats: Optional[torch.Tensor] = None, ln_gamma: Optional[torch.Tensor] = None,
           ln_beta: Optional[torch.Tensor] = None):
    _need_cuda(x.t, y.t, weight, bias, stats)
    _req(weight.dtype == torch.float32 and weight.is_contiguous())
    rc = lib().sdp_dwconv(dcode(x.t.dtype), *x.args(), _ptr(stats), _ptr(ln_gamma), _ptr(ln_beta), weight.data_ptr(),
                          _ptr(bias), *y.args(), B, H, W, C, k, _stream(y.t))
    _check(rc, "dwconv")


def attention(qkv: torch.Tensor, out: torch.Tensor, B: int, N: int, n_head: int, head_dim: int,
              mask: Optional[torch.Tensor] = None, mask_sb: int = 0, mask_sh: int = 0, qk_norm=None,
              eps: float = 1e-5):
    """qk_norm = (q_gamma, q_beta, k_gamma, k_beta) fp32 or None.  NOTE: when the
    generic kernel is taken the norms are applied in place on ``qkv``."""
    _need_cuda(qkv, out, mask)
    _req(qkv.dtype == out.dtype)
    gq, bq, gk, bk = qk_norm if qk_norm is not None else (None, None, None, None)
    rc = lib().sdp_attention(dcode(qkv.dtype), qkv.data_ptr(), qkv.stride(0), out.data_ptr(), out.stride(0), B, N,
                             n_head, head_dim, _ptr(gq), _ptr(bq), _ptr(gk), _ptr(bk), float(eps), _ptr(mask),
                             mask_sb, mask_sh, _stream(out))
    _check(rc, "attention")


def patchify(img: torch.Tensor, out: torch.Tensor, p: int, kpad: int):
    _need_cuda(img, out)
    _req(img.is_contiguous() and img.dim() == 4 and img.shape[1] == 3)
    B, _, Hi, Wi = img.shape
    rc = lib().sdp_patchify(dcode(img.dtype), img.data_ptr(), dcode(out.dtype), out.data_ptr(), B, Hi, Wi, p, kpad,
                            _stream(out))
    _check(rc, "patchify")


def unpatchify(rows: torch.Tensor, img: torch.Tensor, p: int, kpad: int):
    """img [B, 3, Hi, Wi] = the adjoint of patchify applied to rows [B*(Hi/p)*(Wi/p), kpad]."""
    _need_cuda(rows, img)
    _req(img.is_contiguous() and img.dim() == 4 and img.shape[1] == 3 and rows.is_contiguous())
    B, _, Hi, Wi = img.shape
    _req(rows.shape[0] == B * (Hi // p) * (Wi // p) and rows.shape[1] == kpad, "unpatchify rows shape")
    rc = lib().sdp_unpatchify(dcode(rows.dtype), rows.data_ptr(), dcode(img.dtype), img.data_ptr(), B, Hi, Wi, p, kpad,
                              _stream(img))
    _check(rc, "unpatchify")


def pos_table(eh: torch.Tensor, ew: torch.Tensor, out: torch.Tensor, H: int, W: int, C: int):
    _need_cuda(eh, ew, out)
    rc = lib().sdp_pos_table(eh.data_ptr(), ew.data_ptr(), out.data_ptr(), H, W, C, _stream(out))
    _check(rc, "pos_table")


def avgpool_table(bone: torch.Tensor, out: torch.Tensor, H: int, W: int, C: int, k: int):
    _need_cuda(bone, out)
    _req(bone.is_contiguous() and bone.dtype == torch.float32)
    rc = lib().sdp_avgpool_table(bone.data_ptr(), bone.shape[-2], bone.shape[-1], out.data_ptr(), H, W, C, k,
                                 _stream(out))
    _check(rc, "avgpool_table")


def avgpool_table_bwd(dtable: torch.Tensor, dbone: torch.Tensor, H: int, W: int, C: int, k: int):
    """dbone [1, C, BH, BW] fp32 = adjoint of avgpool_table applied to dtable [H*W, C] fp32."""
    _need_cuda(dtable, dbone)
    _req(dtable.is_contiguous() and dbone.is_contiguous() and dtable.dtype == dbone.dtype == torch.float32)
    _req(dtable.numel() >= H * W * C and dbone.shape[-3] == C)
    rc = lib().sdp_avgpool_table_bwd(dtable.data_ptr(), H, W, C, k, dbone.data_ptr(), dbone.shape[-2],
                                     dbone.shape[-1], _stream(dbone))
    _check(rc, "avgpool_table_bwd")


def copy_rows(src: torch.Tensor, lds: int, sgstride: int, dst: torch.Tensor, ldd: int, gstride: int, B: int,
              R: int, C: int, src_offset_rows: int = 0, dst_offset_rows: int = 0):
    _need_cuda(src, dst)
    sp = src.data_ptr() + src_offset_rows * lds * src.element_size()
    dp = dst.data_ptr() + dst_offset_rows * ldd * dst.element_size()
    rc = lib().sdp_copy_rows(dcode(src.dtype), sp, lds, sgstride, dcode(dst.dtype), dp, ldd, gstride, B, R, C,
                             _stream(dst))
    _check(rc, "copy_rows")


def nchw_add_table(x: torch.Tensor, table: torch.Tensor):
    _need_cuda(x, table)
    _req(x.is_contiguous() and table.dtype == torch.float32)
    B, C, H, W = x.shape
    rc = lib().sdp_nchw_add_table(dcode(x.dtype), x.data_ptr(), table.data_ptr(), B, C, H * W, _stream(x))
    _check(rc, "nchw_add_table")


def act(x: torch.Tensor, y: torch.Tensor, code: int):
    _need_cuda(x, y)
    _req(x.is_contiguous() and y.is_contiguous() and x.dtype == y.dtype)
    rc = lib().sdp_act(dcode(x.dtype), x.data_ptr(), y.data_ptr(), x.numel(), code, _stream(y))
    _check(rc, "act")


def group_mean(x: Rows, out: torch.Tensor, G: int, rows: int, C: int):
    _need_cuda(x.t, out)
    rc = lib().sdp_group_mean(dcode(x.t.dtype), *x.args(), dcode(out.dtype), out.data_ptr(), out.stride(0), G, rows,
                              C, _stream(out))
    _check(rc, "group_mean")


def nchw_to_rows(x: torch.Tensor, y: Rows):
    _need_cuda(x, y.t)
    _req(x.is_contiguous())
    B, C, H, W = x.shape
    rc = lib().sdp_nchw_to_rows(dcode(x.dtype), x.data_ptr(), dcode(y.t.dtype), *y.args(), B, C, H * W,
                                _stream(y.t))
    _check(rc, "nchw_to_rows")


def rows_to_nchw(x: Rows, y: torch.Tensor):
    _need_cuda(x.t, y)
    _req(y.is_contiguous())
    B, C, H, W = y.shape
    rc = lib().sdp_rows_to_nchw(dcode(x.t.dtype), *x.args(), dcode(y.dtype), y.data_ptr(), B, C, H * W,
                                _stream(y))
    _check(rc, "rows_to_nchw")


def cast(x: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    _need_cuda(x)
    x = x.contiguous()
    y = torch.empty(x.shape, dtype=dtype, device=x.device)
    rc = lib().sdp_cast(dcode(x.dtype), x.data_ptr(), dcode(dtype), y.data_ptr(), x.numel(), _stream(y))
    _check(rc, "cast")
    return y


def gemm_variant(dtype: torch.dtype, M: int, N: int, K: int) -> int:
    return lib().sdp_gemm_variant(dcode(dtype), M, N, K)


def attention_variant(dtype: torch.dtype, N: int, n_head: int, head_dim: int, has_mask: bool = False) -> int:
    return lib().sdp_attention_variant(dcode(dtype), N, n_head, head_dim, int(has_mask))


def fold_ln_weight(w: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, bias: Optional[torch.Tensor],
                   dtype: torch.dtype):
    """(W * gamma cast to dtype, colsum [N] fp32, beta . W^T + bias [N] fp32) for sdp_gemm_ln."""
    _need_cuda(w, gamma, beta, bias)
    _req(w.dtype == gamma.dtype == beta.dtype == torch.float32 and w.is_contiguous() and w.dim() == 2)
    _req(bias is None or (bias.dtype == torch.float32 and bias.is_contiguous()))
    N, K = w.shape
    wf = torch.empty(N, K, dtype=dtype, device=w.device)
    colsum = torch.empty(N, dtype=torch.float32, device=w.device)
    cvec = torch.empty(N, dtype=torch.float32, device=w.device)
    rc = lib().sdp_fold_ln_weight(w.data_ptr(), gamma.contiguous().data_ptr(), beta.contiguous().data_ptr(),
                                  _ptr(bias), N, K, dcode(dtype), wf.data_ptr(), colsum.data_ptr(), cvec.data_ptr(),
                                  _stream(w))
    _check(rc, "fold_ln_weight")
    return wf, colsum, cvec


def val_preprocess(pix: torch.Tensor, offs: torch.Tensor, hw: torch.Tensor, resize, crop, top: int, left: int,
                   kmax: int, mean, std, tmp_stride: int, dtype: torch.dtype, want_u8: bool = False,
                   max_w: int = 0):
    """Batched validation transform (sdp_val_preprocess); returns (out NCHW, out_u8 or None)."""
    _need_cuda(pix, offs, hw)
    _req(pix.dtype == torch.uint8 and offs.dtype == torch.int64 and hw.dtype == torch.int32)
    B = hw.shape[0]
    (RH, RW), (CH, CW) = resize, crop
    dev = pix.device
    ws = torch.empty(B * (CW + CH) * (2 + kmax), dtype=torch.int32, device=dev)
    tmp = torch.empty(max(1, B * tmp_stride), dtype=torch.uint8, device=dev)
    out = torch.empty(B, 3, CH, CW, dtype=dtype, device=dev)
    u8 = torch.empty(B, CH, CW, 3, dtype=torch.uint8, device=dev) if want_u8 else None
    m3 = (ctypes.c_float * 3)(*[float(v) for v in mean])
    s3 = (ctypes.c_float * 3)(*[float(v) for v in std])
    rc = lib().sdp_val_preprocess(pix.data_ptr(), offs.data_ptr(), hw.data_ptr(), B, RH, RW, top, left, CH, CW,
                                  kmax, m3, s3, ws.data_ptr(), tmp.data_ptr(), tmp_stride, max_w, dcode(dtype),
                                  out.data_ptr(), _ptr(u8), _stream(out))
    _check(rc, "val_preprocess")
    return out, u8


def logits_metrics(logits: torch.Tensor, labels: torch.Tensor, label_smoothing: float = 0.0) -> torch.Tensor:
    """[B, 3] fp32: per-row cross-entropy, BCE-with-logits row sum, top-1 hit."""
    _need_cuda(logits, labels)
    _req(logits.dim() == 2 and logits.stride(1) == 1 and labels.dtype == torch.int64)
    B, C = logits.shape
    labels = labels.contiguous()
    out = torch.empty(B, 3, dtype=torch.float32, device=logits.device)
    rc = lib().sdp_logits_metrics(dcode(logits.dtype), logits.data_ptr(), logits.stride(0), labels.data_ptr(), B, C,
                                  float(label_smoothing), out.data_ptr(), _stream(out))
    _check(rc, "logits_metrics")
    return out


# ---------------------------------------------------------------------------
# training-step kernels (train.hip)
# ---------------------------------------------------------------------------
_NOMAP = [None, 0, 0, 0, 0]


def _rows_args(r: Optional[Rows]):
    return _NOMAP if r is None else r.args()


HIP_ERROR_NOT_SUPPORTED = 801


def gemm_train_epi(mode: int, x: torch.Tensor, w: torch.Tensor, y: torch.Tensor, M: int, N: int, K: int,
                   bias: Optional[torch.Tensor] = None, z: Optional[torch.Tensor] = None,
                   y2: Optional[torch.Tensor] = None, act: int = 0, p: float = 0.0, seed: int = 0) -> bool:
    """Fast-kernel training epilogues (dense bf16 rows): mode 1 y = x w^T + bias, y2 =
    dropout(act(y)); mode 2 y = dropout(x w^T) * act'(z).  False (nothing launched) when the
    fast kernel does not take the shape; the caller then runs gemm + act_fwd / act_bwd."""
    _need_cuda(x, w, y, bias, z, y2)
    _req(x.dtype == w.dtype == y.dtype == torch.bfloat16, "gemm_train_epi bf16 operands")
    _req(all(t.is_contiguous() for t in (x, w, y) + tuple(t for t in (z, y2) if t is not None)))
    _req(x.numel() >= M * K and w.numel() >= N * K and y.numel() >= M * N, "gemm_train_epi operand sizes")
    _req(z is None or (z.dtype == torch.bfloat16 and z.numel() >= M * N), "gemm_train_epi z")
    _req(y2 is None or (y2.dtype == torch.bfloat16 and y2.numel() >= M * N), "gemm_train_epi y2")
    _req(bias is None or (bias.dtype == torch.float32 and bias.numel() >= N), "gemm_train_epi bias fp32")
    rc = lib().sdp_gemm_train_epi(int(mode), x.data_ptr(), K, w.data_ptr(), K, _ptr(bias), _ptr(z), N,
                                  y.data_ptr(), N, _ptr(y2), N, M, N, K, int(act), float(p),
                                  int(seed) & 0xFFFFFFFFFFFFFFFF, _stream(y))
    if rc == HIP_ERROR_NOT_SUPPORTED:
        return False
    _check(rc, "gemm_train_epi")
    return True


def gemm_flex(A: torch.Tensor, B: torch.Tensor, C: torch.Tensor, M: int, N: int, K: int, ta: bool = False,
              tb: bool = False, lda: Optional[int] = None, ldb: Optional[int] = None, ldc: Optional[int] = None,
              Z: int = 1, zdiv: int = 1, sa=(0, 0), sb=(0, 0), sc=(0, 0), splits: int = 1, split_stride: int = 0,
              alpha: float = 1.0, accum: bool = False, a_off: int = 0, b_off: int = 0, c_off: int = 0):
    """C[z](i, j) = alpha * sum_k A(i, k) B(k, j): A(i, k) = A[k, i] if ta else A[i, k];
    B(k, j) = B[j, k] if tb else B[k, j] (row strides lda / ldb / ldc elements, element
    offsets *_off, batch z -> (z // zdiv) * s[0] + (z % zdiv) * s[1])."""
    _need_cuda(A, B, C)
    dt = dcode(A.dtype)
    _req(B.dtype == A.dtype, "gemm_flex operand dtypes")
    od = dcode(C.dtype)
    lda = lda if lda is not None else A.shape[-1]
    ldb = ldb if ldb is not None else B.shape[-1]
    ldc = ldc if ldc is not None else C.shape[-1]
    es, eo = A.element_size(), C.element_size()
    # every element the launch can touch must lie inside the tensors' storage (no OOB launch)
    zmax = lambda s_: ((Z - 1) // zdiv) * s_[0] + min(zdiv - 1, Z - 1) * s_[1]  # noqa: E731
    ar, ac = (K, M) if ta else (M, K)
    br, bc = (N, K) if tb else (K, N)
    for t, off, s_, ld, r, c, what in ((A, a_off, sa, lda, ar, ac, "A"), (B, b_off, sb, ldb, br, bc, "B"),
                                       (C, c_off + (splits - 1) * split_stride, sc, ldc, M, N, "C")):
        if M and N and K and Z:
            last = off + zmax(s_) + (r - 1) * ld + c - 1
            avail = t.untyped_storage().nbytes() // t.element_size() - t.storage_offset()
            _req(0 <= off and c <= ld and last < avail, f"gemm_flex operand {what} out of bounds")
    rc = lib().sdp_gemm_flex(dt, od, int(ta), int(tb), A.data_ptr() + a_off * es, lda, sa[0], sa[1],
                             B.data_ptr() + b_off * es, ldb, sb[0], sb[1], C.data_ptr() + c_off * eo, ldc, sc[0],
                             sc[1], M, N, K, Z, zdiv, splits, split_stride, float(alpha), int(bool(accum)), _stream(C))
    _check(rc, "gemm_flex")


def mt_cast_transpose(jobs):
    """jobs: [(src fp32 [R, C] contiguous, dst bf16 view or None, dstT bf16 view or None)]:
    dst[r, c] = bf16(src[r, c]) and dstT[c, r] = bf16(src[r, c]) in one launch (dst / dstT may be
    row-strided views; unit column stride)."""
    import struct
    if not jobs:
        return
    dev = jobs[0][0].device
    eb = lib().sdp_mt_cast_transpose_entry_bytes()
    raw, tiles = bytearray(), []
    for i, (src, dst, dt_) in enumerate(jobs):
        _need_cuda(src, dst, dt_)
        _req(src.dtype == torch.float32 and src.dim() == 2 and src.is_contiguous(), "mt_cast_transpose src")
        R, C = src.shape
        for t, shp in ((dst, (R, C)), (dt_, (C, R))):
            _req(t is None or (t.dtype == torch.bfloat16 and tuple(t.shape) == shp and t.stride(1) == 1),
                 "mt_cast_transpose outputs")
        ent = struct.pack("<QQQqqii", src.data_ptr(), 0 if dst is None else dst.data_ptr(),
                          0 if dt_ is None else dt_.data_ptr(), 0 if dst is None else dst.stride(0),
                          0 if dt_ is None else dt_.stride(0), R, C)
        raw += ent + bytes(eb - len(ent))
        tiles += [(i, r0, c0, 0) for r0 in range(0, R, 64) for c0 in range(0, C, 64)]
    ent = torch.frombuffer(raw, dtype=torch.uint8).to(dev)
    tl = torch.tensor(tiles, dtype=torch.int32, device=dev)
    _check(lib().sdp_mt_cast_transpose(ent.data_ptr(), tl.data_ptr(), len(tiles), _stream(jobs[0][0])),
           "mt_cast_transpose")


_ZERO_ROWS = {}


def _zero_row(device, n: int) -> torch.Tensor:
    """A cached zero bf16 row of >= n elements (the rows gemm_wgrad reads past the last token)."""
    key = (str(device), torch.cuda.current_stream(device).cuda_stream)
    z = _ZERO_ROWS.get(key)
    if z is None or z.numel() < n:
        z = torch.zeros(max(n, 4096), dtype=torch.bfloat16, device=device)
        # inside a graph capture the zeros are a memset node that only runs on replay: such a
        # buffer is valid for that graph alone, so it is not cached for eager launches
        if not torch.cuda.is_current_stream_capturing():
            _ZERO_ROWS[key] = z
    return z


def gemm_wgrad(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor, ktok: int, kchunk_tiles: int,
               split_stride: int = 0):
    """out[s] (fp32 [N, K] slabs) = dy[rows of split s]^T x[rows of split s] on the 8-phase MFMA
    kernel (sdp_gemm_wgrad); dy [>= ktok, N], x [>= ktok, K] bf16 with unit column stride."""
    _need_cuda(dy, x, out)
    _req(dy.dtype == x.dtype == torch.bfloat16 and out.dtype == torch.float32, "gemm_wgrad dtypes")
    _req(dy.stride(1) == 1 and x.stride(1) == 1 and out.stride(-1) == 1, "gemm_wgrad unit column strides")
    N, K = dy.shape[1], x.shape[1]
    _req(dy.shape[0] >= ktok and x.shape[0] >= ktok and ktok > 0, "gemm_wgrad token rows")
    nkt = (ktok + 63) // 64
    zrow = _zero_row(dy.device, max(N, K)) if ktok % 64 else None
    splits = (nkt + kchunk_tiles - 1) // kchunk_tiles
    ldc = out.stride(-2)
    _req(out.shape[-2] >= N and out.shape[-1] >= K, "gemm_wgrad output shape")
    last = (splits - 1) * split_stride + (N - 1) * ldc + K
    avail = out.untyped_storage().nbytes() // 4 - out.storage_offset()
    _req(last <= avail and (splits == 1 or split_stride >= N * ldc), "gemm_wgrad output out of bounds")
    rc = lib().sdp_gemm_wgrad(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), out.data_ptr(), ldc,
                              split_stride, N, K, ktok, kchunk_tiles, _ptr(zrow), _stream(out))
    _check(rc, "gemm_wgrad")


def seg_colsum(X: torch.Tensor, out: torch.Tensor, G: int, length: int, gstride: int, estride: int, C: int,
               ldx: Optional[int] = None, ldo: Optional[int] = None, scale: float = 1.0, accum: bool = False,
               x_off: int = 0):
    """out[g, c] (+)= scale * sum_e X[(g * gstride + e * estride) * ldx + x_off + c] (fp32 out)."""
    _need_cuda(X, out)
    _req(out.dtype == torch.float32, "seg_colsum out fp32")
    ldx = ldx if ldx is not None else X.shape[-1]
    ldo = ldo if ldo is not None else C
    rc = lib().sdp_seg_colsum(dcode(X.dtype), X.data_ptr() + x_off * X.element_size(), ldx, G, length, gstride,
                              estride, C, out.data_ptr(), ldo, float(scale), int(bool(accum)), _stream(out))
    _check(rc, "seg_colsum")


def act_fwd(Z: torch.Tensor, Y: torch.Tensor, M: int, N: int, code: int, p: float = 0.0, seed: int = 0,
            ldz: Optional[int] = None, ldy: Optional[int] = None):
    _need_cuda(Z, Y)
    _req(Z.dtype == Y.dtype, "act_fwd dtypes")
    rc = lib().sdp_act_fwd(dcode(Z.dtype), Z.data_ptr(), ldz or N, Y.data_ptr(), ldy or N, M, N, code, float(p),
                           int(seed) & 0xFFFFFFFFFFFFFFFF, _stream(Y))
    _check(rc, "act_fwd")


def act_bwd(Z: torch.Tensor, DY: torch.Tensor, DZ: torch.Tensor, M: int, N: int, code: int, p: float = 0.0,
            seed: int = 0, ld: Optional[int] = None):
    """ld: the row stride of Z, DY and DZ (default N)."""
    _need_cuda(Z, DY, DZ)
    _req(Z.dtype == DY.dtype == DZ.dtype, "act_bwd dtypes")
    ld = ld or N
    rc = lib().sdp_act_bwd(dcode(Z.dtype), Z.data_ptr(), ld, DY.data_ptr(), ld, DZ.data_ptr(), ld, M, N, code, float(p),
                           int(seed) & 0xFFFFFFFFFFFFFFFF, _stream(DZ))
    _check(rc, "act_bwd")


def rowscale_add(x: Rows, y: Rows, M: int, N: int, scale: Optional[torch.Tensor] = None, sgrp: int = 1,
                 resid: Optional[Rows] = None, act: int = 0, p: float = 0.0, seed: int = 0, dmode: int = 0):
    """y = act(x) * scale[m / sgrp] (+ resid) over row maps (act 0: sdp_rowscale_add).  x may
    differ in dtype from y (resid has y's dtype): sdp_rowscale_add_mixed.  p > 0 with dmode 1 /
    2: dropout (counter hash, index m * N + n) on x / on the rounded output
    (sdp_rowscale_add_dropout; act must be 0)."""
    _need_cuda(x.t, y.t, scale)
    _req(scale is None or scale.dtype == torch.float32, "rowscale scale fp32")
    _req(resid is None or resid.t.dtype == y.t.dtype, "rowscale resid dtype = y dtype")
    if p > 0 and dmode:
        _req(act == 0 and dmode in (1, 2), "rowscale dropout: no activation, mode 1 or 2")
        rc = lib().sdp_rowscale_add_dropout(dcode(x.t.dtype), dcode(y.t.dtype), *x.args(), _ptr(scale), sgrp,
                                            *_rows_args(resid), *y.args(), M, N, float(p),
                                            int(seed) & 0xFFFFFFFFFFFFFFFF, int(dmode), _stream(y.t))
        if rc != _HIP_NOT_SUPPORTED:
            _check(rc, "rowscale_add_dropout")
            return
        # unaligned rows / N % 8 != 0: the same arithmetic as two passes (dense operands only)
        _req(x.t.is_contiguous() and x.t.shape[-1] == N and y.t.is_contiguous() and y.t.shape[-1] == N,
             "rowscale dropout fallback: dense rows")
        if dmode == 1:
            tmp = torch.empty(M, N, dtype=x.t.dtype, device=x.t.device)
            act_fwd(x.t, tmp, M, N, 0, p, seed)
            rowscale_add(Rows(tmp, N), y, M, N, scale=scale, sgrp=sgrp, resid=resid)
        else:
            rowscale_add(x, y, M, N, scale=scale, sgrp=sgrp, resid=resid)
            act_bwd(y.t, y.t, y.t, M, N, 0, p, seed)
        return
    if x.t.dtype != y.t.dtype:
        rc = lib().sdp_rowscale_add_mixed(dcode(x.t.dtype), dcode(y.t.dtype), int(act), *x.args(), _ptr(scale), sgrp,
                                          *_rows_args(resid), *y.args(), M, N, _stream(y.t))
    elif act:
        rc = lib().sdp_act_rowscale_add(dcode(x.t.dtype), int(act), *x.args(), _ptr(scale), sgrp, *_rows_args(resid),
                                        *y.args(), M, N, _stream(y.t))
    else:
        rc = lib().sdp_rowscale_add(dcode(x.t.dtype), *x.args(), _ptr(scale), sgrp, *_rows_args(resid), *y.args(), M,
                                    N, _stream(y.t))
    _check(rc, "rowscale_add")


def add_ln_fwd(x: Rows, y: Rows, a: Rows, M: int, C: int, resid: Rows, eps: float, gamma: torch.Tensor,
               beta: torch.Tensor, stats: torch.Tensor, scale: Optional[torch.Tensor] = None, sgrp: int = 1,
               act: int = 0, p: float = 0.0, seed: int = 0, dmode: int = 0, regs=None) -> bool:
    """y = act / dropout(x) * scale[m / sgrp] + resid and a = LN(y) (+ its statistics) in one pass
    (sdp_add_ln_fwd; bit-identical to rowscale_add followed by ln_fwd).  regs = (src, [dst0, dst1], B, R,
    N): also copy the register rows (token buffers [B, N, C] in y's dtype) in the same launch.  False
    where the one-pass form does not apply (the caller runs the two passes and the copies)."""
    _need_cuda(x.t, y.t, a.t, resid.t, gamma, beta, stats, scale)
    _req(resid.t.dtype == y.t.dtype, "add_ln_fwd: resid dtype = y dtype")
    _req(stats.dtype == gamma.dtype == beta.dtype == torch.float32, "add_ln_fwd fp32 params")
    _req(scale is None or scale.dtype == torch.float32, "add_ln_fwd scale fp32")
    rsrc, rd0, rd1, rb, rr, rn = _reg_args(regs, y.t.dtype, C, 2)
    rc = lib().sdp_add_ln_fwd(dcode(x.t.dtype), dcode(y.t.dtype), dcode(a.t.dtype), int(act), *x.args(), _ptr(scale),
                              sgrp, *resid.args(), *y.args(), float(p), int(seed) & 0xFFFFFFFFFFFFFFFF, int(dmode),
                              float(eps), gamma.data_ptr(), beta.data_ptr(), stats.data_ptr(), *a.args(), M, C,
                              rsrc, rd0, rd1, rb, rr, rn, _stream(y.t))
    if rc == _HIP_NOT_SUPPORTED:
        return False
    _check(rc, "add_ln_fwd")
    return True


def _reg_args(regs, dt, C: int, ndst: int):
    """(src ptr, dst0, dst1, B, R, N) of a register-row copy job regs = (src, [dsts], B, R, N), or Nones."""
    if regs is None:
        return None, None, None, 0, 0, 0
    src, dsts, B, R, N = regs
    _req(1 <= len(dsts) <= ndst, "register copy: destinations")
    for t in (src, *dsts):
        _need_cuda(t)
        _req(t.dtype == dt and t.is_contiguous() and t.numel() >= B * N * C and t.shape[-1] == C and R <= N,
             "register copy operands")
    return (src.data_ptr(), dsts[0].data_ptr(), dsts[1].data_ptr() if len(dsts) > 1 else None, int(B), int(R),
            int(N))


def copy_regs(regs):
    """The register-row copy job of regs = (src, [dsts], B, R, N) as separate copy_rows launches."""
    if regs is None:
        return
    src, dsts, B, R, N = regs
    C = src.shape[-1]
    if R:
        for d in dsts:
            copy_rows(src, C, N * C, d, C, N * C, B, R, C)


def ln_apply(x: Rows, stats: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, y: Rows, M: int, C: int):
    _need_cuda(x.t, y.t, stats, gamma, beta)
    _req(stats.dtype == gamma.dtype == beta.dtype == torch.float32, "ln_apply fp32 params")
    rc = lib().sdp_ln_apply(dcode(x.t.dtype), *x.args(), stats.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                            *y.args(), M, C, _stream(y.t))
    _check(rc, "ln_apply")


_TICKETS = {}
# SDPNET_LN_BWD_FUSED=0: LayerNorm backward as before (partials + two seg_colsum launches, branch passes
# separate) -- A/B switch
_LN_BWD_FUSED = os.environ.get("SDPNET_LN_BWD_FUSED", "1") != "0"
# SDPNET_LN_TICKET=1: the affine sums finished inside the LayerNorm backward (ticketed last-block
# reduction; its device-scope fences measured far slower on the XL training step), else the two
# seg_colsum levels after it
_LN_TICKET = os.environ.get("SDPNET_LN_TICKET", "0") != "0"


def _tickets(dev: torch.device) -> torch.Tensor:
    """Zeroed ints for the in-kernel affine sums of sdp_ln_bwd_fused, one buffer per (device,
    stream): the kernels leave them zeroed, and launches on one stream never overlap."""
    st = torch.cuda.current_stream(dev)
    key = (dev.index, st.cuda_stream)
    t = _TICKETS.get(key)
    if t is None:
        t = _TICKETS[key] = torch.zeros(64, dtype=torch.int32, device=dev)
    return t


def ln_bwd(x: Rows, stats: torch.Tensor, gamma: torch.Tensor, dy: Rows, dx: Rows, M: int, C: int,
           add: Optional[Rows] = None, want_affine: bool = True, emit: Optional[dict] = None, regs=None):
    """dx (= LN backward [+ add]); returns (dgamma, dbeta) fp32 [C] or None.

    emit = dict(out=bf16 [M, C] dense, scale=None, sgrp=1, z=None, act=0, p=0.0, seed=0, dmode=0): also
    writes the gradient of the branch that fed the LayerNorm input, as sdp_rowscale_add (scale, and
    dmode 2 dropout) followed by sdp_act_bwd (act'(z)) would from the stored dx -- in the same launch
    where sdp_ln_bwd_fused applies, else by those two passes (bit-identical either way).
    regs = (src, [dst], B, R, N): register rows of src (dx's dtype) copied to dst, in the same launch
    where it applies."""
    _need_cuda(x.t, stats, gamma, dy.t, dx.t)
    _req(dx.t.dtype == x.t.dtype and (add is None or add.t.dtype == x.t.dtype), "ln_bwd x / add / dx dtypes")
    nb = lib().sdp_ln_bwd_blocks(M)
    dev = dx.t.device
    part = torch.empty(nb, 2, C, dtype=torch.float32, device=dev) if want_affine else None
    if emit is not None:
        o2, z = emit["out"], emit.get("z")
        _need_cuda(o2, z, emit.get("scale"))
        _req(o2.dtype == torch.bfloat16 and o2.is_contiguous() and o2.shape[0] >= M and o2.shape[-1] == C and
             (z is None or (z.dtype == torch.bfloat16 and z.is_contiguous() and z.shape[0] >= M and z.shape[-1] == C)),
             "ln_bwd emit operands")
    ticket = want_affine and _LN_TICKET
    rsrc, rd0, _, rb, rr, rn = _reg_args(regs, dx.t.dtype, C, 1)
    if _LN_BWD_FUSED and M > 0 and (emit is not None or ticket or regs is not None):
        ng = (nb + 31) // 32
        gpart = torch.empty(ng, 2 * C, dtype=torch.float32, device=dev) if ticket else None
        aff = torch.empty(2 * C, dtype=torch.float32, device=dev) if ticket else None
        e = emit or {}
        sc = e.get("scale")
        rc = lib().sdp_ln_bwd_fused(dcode(x.t.dtype), dcode(dy.t.dtype), *x.args(), stats.data_ptr(), gamma.data_ptr(),
                                    *dy.args(), *_rows_args(add), *dx.args(), M, C, _ptr(part), _ptr(gpart), _ptr(aff),
                                    _tickets(dev).data_ptr() if ticket else None, _ptr(sc), int(e.get("sgrp", 1)),
                                    _ptr(e.get("z")), C, int(e.get("act", 0)), float(e.get("p", 0.0)),
                                    int(e.get("seed", 0)) & 0xFFFFFFFFFFFFFFFF, int(e.get("dmode", 0)),
                                    _ptr(e.get("out")), C, rsrc, rd0, rb, rr, rn, _stream(dx.t))
        if rc != _HIP_NOT_SUPPORTED:
            _check(rc, "ln_bwd_fused")
            if ticket:
                return aff[:C], aff[C:]
            return _affine_sums(part, nb, C) if want_affine else None
    copy_regs(regs)
    if dy.t.dtype != x.t.dtype:  # fp32 stream, bf16 gradient of the LN output
        rc = lib().sdp_ln_bwd_mixed(dcode(x.t.dtype), dcode(dy.t.dtype), *x.args(), stats.data_ptr(), gamma.data_ptr(),
                                    *dy.args(), *_rows_args(add), *dx.args(), M, C, _ptr(part), _stream(dx.t))
    else:
        rc = lib().sdp_ln_bwd(dcode(x.t.dtype), *x.args(), stats.data_ptr(), gamma.data_ptr(), *dy.args(),
                              *_rows_args(add), *dx.args(), M, C, _ptr(part), _stream(dx.t))
    _check(rc, "ln_bwd")
    if emit is not None:  # the two passes the one-launch form replaces
        o2, z = emit["out"], emit.get("z")
        rowscale_add(dx, dense(o2[:M]) if o2.shape[0] != M else dense(o2), M, C, scale=emit.get("scale"),
                     sgrp=int(emit.get("sgrp", 1)), p=float(emit.get("p", 0.0)), seed=int(emit.get("seed", 0)),
                     dmode=int(emit.get("dmode", 0)))
        if int(emit.get("act", 0)):
            act_bwd(z[:M], o2[:M], o2[:M], M, C, int(emit["act"]))
    if part is None:
        return None
    return _affine_sums(part, nb, C)


def _affine_sums(part: torch.Tensor, nb: int, C: int):
    """(dgamma, dbeta) from the LayerNorm backward's per-block partials [nb, 2, C]."""
    dev = part.device
    out = torch.empty(2, C, dtype=torch.float32, device=dev)
    if nb >= 128:  # two levels: 32-row chunk sums in parallel, then the chunk sums
        g = nb // 32
        tmp = torch.empty(g + 1, 2 * C, dtype=torch.float32, device=dev)
        seg_colsum(part.view(nb, 2 * C), tmp, g, 32, 32, 1, 2 * C)
        rest = nb - 32 * g
        if rest:
            seg_colsum(part.view(nb, 2 * C), tmp[g:], 1, rest, 0, 1, 2 * C, x_off=32 * g * 2 * C)
        seg_colsum(tmp, out.view(1, 2 * C), 1, g + (1 if rest else 0), 0, 1, 2 * C)
    else:
        seg_colsum(part.view(nb, 2 * C), out.view(1, 2 * C), 1, nb, 0, 1, 2 * C)
    return out[0], out[1]


def softmax_fwd(S: torch.Tensor, P: torch.Tensor, Pd: Optional[torch.Tensor], rows: int, N: int, Npad: int,
                scale: float, p: float = 0.0, seed: int = 0, mask: Optional[Tuple[torch.Tensor, int, int, int]] = None):
    """mask = (additive fp32 bias, batch stride, head stride, heads): bias[(z // heads) * sb +
    (z % heads) * sh + i * N + c] is added to row z * N + i before the softmax."""
    _need_cuda(S, P, Pd)
    _req(S.dtype == torch.float32, "softmax S fp32")
    if mask is None:
        rc = lib().sdp_softmax_fwd(dcode(P.dtype), S.data_ptr(), S.shape[-1], P.data_ptr(), _ptr(Pd), P.shape[-1],
                                   rows, N, Npad, float(scale), float(p), int(seed) & 0xFFFFFFFFFFFFFFFF, _stream(P))
    else:
        mb, sb, sh, zdiv = mask
        _need_cuda(mb)
        Z = rows // N
        last = ((Z - 1) // zdiv) * sb + min(zdiv - 1, Z - 1) * sh + (N - 1) * N + N - 1
        _req(mb.dtype == torch.float32 and rows % N == 0 and sb >= 0 and sh >= 0 and
             last < mb.untyped_storage().nbytes() // 4 - mb.storage_offset(), "softmax mask bounds")
        rc = lib().sdp_softmax_fwd_mask(dcode(P.dtype), S.data_ptr(), S.shape[-1], P.data_ptr(), _ptr(Pd),
                                        P.shape[-1], rows, N, Npad, float(scale), float(p),
                                        int(seed) & 0xFFFFFFFFFFFFFFFF, mb.data_ptr(), sb, sh, zdiv, _stream(P))
    _check(rc, "softmax_fwd")


def softmax_bwd(P: torch.Tensor, dPd: torch.Tensor, dS: torch.Tensor, rows: int, N: int, Npad: int, p: float = 0.0,
                seed: int = 0):
    _need_cuda(P, dPd, dS)
    rc = lib().sdp_softmax_bwd(dcode(P.dtype), P.data_ptr(), P.shape[-1], dPd.data_ptr(), dPd.shape[-1],
                               dS.data_ptr(), dS.shape[-1], rows, N, Npad, float(p), int(seed) & 0xFFFFFFFFFFFFFFFF,
                               _stream(dS))
    _check(rc, "softmax_bwd")


def dw_wgrad(a: Rows, dy: Rows, B: int, H: int, W: int, C: int, k: int) -> torch.Tensor:
    """Depthwise weight gradient [C, k*k] fp32 (reduced over the chunk slabs)."""
    _need_cuda(a.t, dy.t)
    nch = lib().sdp_dw_wgrad_chunks(B)
    part = torch.empty(nch, C * k * k, dtype=torch.float32, device=a.t.device)
    rc = lib().sdp_dw_wgrad(dcode(a.t.dtype), *a.args(), *dy.args(), B, H, W, C, k, part.data_ptr(), _stream(part))
    _check(rc, "dw_wgrad")
    out = torch.empty(C, k * k, dtype=torch.float32, device=a.t.device)
    seg_colsum(part, out.view(1, -1), 1, nch, 0, 1, C * k * k)
    return out


def ce_loss(logits: torch.Tensor, labels: torch.Tensor, eps: float, grad_scale: float,
            dlogits: Optional[torch.Tensor], loss: torch.Tensor, ignore_index: int = -100):
    """Label-smoothed CE, mean over the rows whose label != ignore_index (those get zero dlogits)."""
    _need_cuda(logits, labels, dlogits, loss)
    _req(labels.dtype == torch.int64 and loss.dtype == torch.float32, "ce_loss dtypes")
    B, K = logits.shape
    _req(labels.numel() == B, "ce_loss: one label per row")
    labels = labels.contiguous()
    nrows = torch.empty(1, dtype=torch.float32, device=loss.device)
    _check(lib().sdp_ce_count(labels.data_ptr(), B, int(ignore_index), nrows.data_ptr(), _stream(loss)), "ce_count")
    rc = lib().sdp_ce_loss_counted(dcode(logits.dtype), logits.data_ptr(), logits.stride(0),
                                   labels.data_ptr(), B, K, float(eps), float(grad_scale),
                                   int(ignore_index), nrows.data_ptr(), _ptr(dlogits),
                                   dlogits.stride(0) if dlogits is not None else 0, loss.data_ptr(), _stream(loss))
    _check(rc, "ce_loss")


def ce_loss_soft(logits: torch.Tensor, targets: torch.Tensor, eps: float, grad_scale: float,
                 dlogits: Optional[torch.Tensor], loss: torch.Tensor):
    """Cross entropy on probability targets [B, K] fp32 (nn.CrossEntropyLoss with soft targets)."""
    _need_cuda(logits, targets, dlogits, loss)
    _req(targets.dtype == torch.float32 and loss.dtype == torch.float32 and targets.shape == logits.shape
         and targets.stride(1) == 1, "ce_loss_soft: fp32 [B, K] targets")
    B, K = logits.shape
    rc = lib().sdp_ce_loss_soft(dcode(logits.dtype), logits.data_ptr(), logits.stride(0), targets.data_ptr(),
                                targets.stride(0), B, K, float(eps), float(grad_scale), _ptr(dlogits),
                                dlogits.stride(0) if dlogits is not None else 0, loss.data_ptr(), _stream(loss))
    _check(rc, "ce_loss_soft")


def transpose(x: torch.Tensor) -> torch.Tensor:
    """x [R, C] (row stride x.stride(0)) -> contiguous [C, R] on the HIP transpose kernel."""
    _need_cuda(x)
    _req(x.dim() == 2 and x.stride(1) == 1, "transpose of a row-major 2-D tensor")
    R, C = x.shape
    y = torch.empty(C, R, dtype=x.dtype, device=x.device)
    rc = lib().sdp_transpose(dcode(x.dtype), x.data_ptr(), x.stride(0), y.data_ptr(), R, R, C, _stream(y))
    _check(rc, "transpose")
    return y


def ln_fwd(x: Rows, eps: float, gamma: torch.Tensor, beta: torch.Tensor, stats: torch.Tensor, y: Rows, M: int, C: int):
    """One-pass LayerNorm that also writes its (mean, rstd) statistics (training forward)."""
    _need_cuda(x.t, y.t, gamma, beta, stats)
    _req(stats.dtype == gamma.dtype == beta.dtype == torch.float32, "ln_fwd fp32 params")
    if x.t.dtype != y.t.dtype:
        rc = lib().sdp_ln_fwd_mixed(dcode(x.t.dtype), dcode(y.t.dtype), *x.args(), float(eps), gamma.data_ptr(),
                                    beta.data_ptr(), stats.data_ptr(), *y.args(), M, C, _stream(y.t))
    else:
        rc = lib().sdp_ln_fwd(dcode(x.t.dtype), *x.args(), float(eps), gamma.data_ptr(), beta.data_ptr(),
                              stats.data_ptr(), *y.args(), M, C, _stream(y.t))
    _check(rc, "ln_fwd")


# ------------------------------------------------------------------ flash training attention
def attn_train_applies(dtype: torch.dtype, N: int, hd: int) -> bool:
    return dtype == torch.bfloat16 and bool(lib().sdp_attn_train_applies(BF16, N, hd))


def attn_train_fwd(qkv: torch.Tensor, o: torch.Tensor, lse: torch.Tensor, B: int, N: int, H: int, hd: int,
                   scale: float, p: float, seed: int):
    """O = dropout(softmax(scale Q K^T)) V (rows of o), lse (fp32, B*H*N) = base-2 log-sum-exp."""
    _need_cuda(qkv, o, lse)
    _req(qkv.dtype == o.dtype == torch.bfloat16 and lse.dtype == torch.float32 and lse.numel() >= B * H * N)
    _req(qkv.shape[0] >= B * N and o.shape[0] >= B * N and qkv.stride(1) == 1 and o.stride(1) == 1)
    rc = lib().sdp_attn_train_fwd(BF16, qkv.data_ptr(), qkv.stride(0), o.data_ptr(), o.stride(0), lse.data_ptr(),
                                  B, N, H, hd, float(scale), float(p), int(seed) & 0xFFFFFFFFFFFFFFFF, _stream(o))
    _check(rc, "attn_train_fwd")


def attn_train_bwd(qkv: torch.Tensor, o: torch.Tensor, do: torch.Tensor, lse: torch.Tensor, delta: torch.Tensor,
                   dq: Tuple[torch.Tensor, int], dk: Tuple[torch.Tensor, int], dv: Tuple[torch.Tensor, int],
                   B: int, N: int, H: int, hd: int, scale: float, p: float, seed: int):
    """dQ, dK, dV into (tensor, first column) row blocks; delta: fp32 scratch of B*H*N."""
    _need_cuda(qkv, o, do, lse, delta, dq[0], dk[0], dv[0])
    _req(qkv.dtype == o.dtype == do.dtype == torch.bfloat16 and delta.numel() >= B * H * N)
    for t, c in (dq, dk, dv):
        _req(t.dtype == torch.bfloat16 and t.stride(1) == 1 and t.shape[0] >= B * N and t.shape[1] >= c + H * hd)
    es = 2
    rc = lib().sdp_attn_train_bwd(BF16, qkv.data_ptr(), qkv.stride(0), o.data_ptr(), o.stride(0), do.data_ptr(),
                                  do.stride(0), lse.data_ptr(), delta.data_ptr(),
                                  dq[0].data_ptr() + es * dq[1], dq[0].stride(0),
                                  dk[0].data_ptr() + es * dk[1], dk[0].stride(0),
                                  dv[0].data_ptr() + es * dv[1], dv[0].stride(0),
                                  B, N, H, hd, float(scale), float(p), int(seed) & 0xFFFFFFFFFFFFFFFF, _stream(o))
    _check(rc, "attn_train_bwd")


def attn_dropout_mask(Z: int, N: int, p: float, seed: int, device) -> torch.Tensor:
    """The training attention's dropout keep mask [Z, N, N] (uint8, 1 = kept), for tests."""
    out = torch.empty(Z, N, N, dtype=torch.uint8, device=device)
    _check(lib().sdp_attn_dropout_mask(out.data_ptr(), Z, N, float(p), int(seed) & 0xFFFFFFFFFFFFFFFF, _stream(out)),
           "attn_dropout_mask")
    return out
