"""CPU: the C-ABI library loads and exports every symbol include/sdpnet_hip.h
declares, and its host-side argument validation works (no kernel launches)."""
import ctypes
import os
import re

import pytest
import torch  # noqa: F401  (load torch's HIP runtime first, as the product does)

import sdpnet_hip as sp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "sdpnet_hip.h")


def header_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int64_t|int|const char\*)\s+(sdp_\w+)\s*\(", src, re.M)))


def test_library_exports_every_header_symbol():
    L = sp.lib()
    syms = header_symbols()
    assert len(syms) >= 18
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(sp.exported_symbols()) == syms


def test_version_string():
    assert b"gfx950" in sp.lib().sdp_version()


def test_gemm_variant_selection():
    L = sp.lib()
    assert L.sdp_gemm_variant(1, 50176, 768, 768) == 1
    assert L.sdp_gemm_variant(1, 51200, 3072, 768) == 1
    assert L.sdp_gemm_variant(1, 256, 1000, 1000) == 0   # K % 64 != 0 -> generic
    assert L.sdp_gemm_variant(0, 50176, 768, 768) == 0   # fp32 -> exact f32 MFMA generic


def test_attention_variant_selection():
    L = sp.lib()
    assert L.sdp_attention_variant(1, 200, 8, 96, 0) == 4   # M: two persistent workgroups per CU
    assert L.sdp_attention_variant(1, 260, 8, 96, 0) == 3   # XL: whole head staged
    assert L.sdp_attention_variant(1, 1000, 8, 96, 0) == 5  # long heads: streamed K / V
    old = L.sdp_attention_set_kernel(6)  # attn_fa5 (slower in the model): diagnostic build only
    if L.sdp_build_info() == 0:
        assert old == -1 and L.sdp_attention_set_kernel(0) == 4  # refused, selection unchanged
    else:
        try:
            assert L.sdp_attention_variant(1, 200, 8, 96, 0) == 6
            assert L.sdp_attention_variant(1, 240, 8, 96, 0) == 4   # N > 224 -> fa4
            assert L.sdp_attention_variant(1, 200, 4, 128, 0) == 4  # fa5's double buffer exceeds 160 KiB
        finally:
            L.sdp_attention_set_kernel(old)
    assert L.sdp_attention_variant(1, 200, 8, 96, 1) == 0   # masks -> generic
    assert L.sdp_attention_variant(0, 200, 8, 96, 0) == 0   # fp32 -> generic
    assert L.sdp_attention_variant(1, 53, 8, 12, 0) == 0    # hd % 8 != 0


def test_invalid_arguments_rejected_before_launch():
    L = sp.lib()
    # null operands -> hipErrorInvalidValue (1), no device touched
    assert L.sdp_gemm(1, None, 64, 0, 0, 0, None, 64, None, None, 0, 0, 0, 0, None, 64, 0, 0, 0,
                      128, 128, 64, 0, 0, None) == 1
    assert L.sdp_layernorm(1, None, 8, 0, 0, 0, None, None, 1e-5, None, 8, 0, 0, 0, 4, 8, None) == 1
    assert L.sdp_attention(1, None, 8, None, 8, 1, 4, 1, 8, None, None, None, None, 1e-5, None, 0, 0, None) == 1
    assert L.sdp_patchify(0, None, 1, None, 1, 224, 224, 16, 768, None) == 1
    assert L.sdp_cast(0, None, 1, None, 10, None) == 1
    # degenerate sizes are no-ops
    assert L.sdp_gemm(1, 8, 64, 0, 0, 0, 8, 64, None, None, 0, 0, 0, 0, 8, 64, 0, 0, 0,
                      0, 128, 64, 0, 0, None) == 0


def test_wrapper_rejects_cpu_tensors():
    x = torch.zeros(4, 8)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        sp.layernorm(sp.dense(x), torch.ones(8), torch.zeros(8), 1e-5, sp.dense(x), 4, 8)


def test_product_library_has_no_kernel_skip_paths():
    """The product library compiles the timing-experiment skips out (SDP_DIAG only): a
    non-zero request is refused and the mask stays 0, and sdp_build_info() reports 0."""
    L = sp.lib()
    assert L.sdp_build_info() == 0
    assert L.sdp_debug_skip(3) == -1
    assert L.sdp_debug_skip(0) == 0


class _FakeLib:
    def __init__(self, info=0, mask=0):
        self.info, self.mask = info, mask

    def sdp_build_info(self):
        return self.info

    def sdp_debug_skip(self, m):
        old, self.mask = self.mask, m
        return old


def test_bench_refuses_skip_masks_and_diagnostic_builds():
    """bench.py's integrity gate: a diagnostic library, a non-zero skip mask or SDPNET_DEBUG_SKIP
    make it exit before timing; otherwise it returns the SDPNET_* knobs it records."""
    import sys
    sys.path.insert(0, REPO)
    import bench
    assert bench.check_library(_FakeLib(), {"PATH": "/bin"}) == {}
    assert bench.check_library(_FakeLib(), {"SDPNET_STREAMS": "2", "X": "1"}) == {"SDPNET_STREAMS": "2"}
    with pytest.raises(SystemExit, match="diagnostic"):
        bench.check_library(_FakeLib(info=1), {})
    with pytest.raises(SystemExit, match="skip"):
        bench.check_library(_FakeLib(mask=2), {})
    with pytest.raises(SystemExit, match="skip"):
        bench.check_library(_FakeLib(), {"SDPNET_DEBUG_SKIP": "1"})
    # the real product library passes the gate
    assert bench.check_library(sp.lib(), {}) == {}
