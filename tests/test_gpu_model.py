"""GPU: the drop-in model on the HIP path against the reference's golden logits
(made by the reference itself, tests/golden/) and against the CPU oracle.

Tolerances (BASELINE.json north_star): fp32 logits within 1e-3 absolute of the
reference fp32 CPU forward; bf16 within 1e-2 absolute.  Full-size (bs=256)
behaviour is checked through size-independent properties: per-image results do
not depend on the batch they run in (bit-exact), and are finite.
"""
import numpy as np
import pytest
import torch

import golden_util as gu
import sdpnet_oracle as orc
import synth

pytestmark = pytest.mark.gpu
DEV = "cuda"
FP32_TOL = 1e-3
BF16_TOL = 1e-2

_MODELS = {}


def get_model(name):
    """(model on GPU in eval mode, meta, arrays, x) for a golden case; cached."""
    if name not in _MODELS:
        import model as ours
        meta, arr = gu.load_case(name)
        torch.manual_seed(0)
        m = ours.MainModel.from_dict(**meta["config"])
        sd, x = gu.build_inputs(meta, m)
        assert gu.digest(sd) == meta["weights_sha256"]
        m.load_state_dict(sd)
        m = m.to(DEV).eval()
        _MODELS.clear()
        _MODELS[name] = (m, meta, arr, x)
    return _MODELS[name]


CASES = gu.case_names()


@pytest.mark.parametrize("name", CASES)
def test_fp32_logits_match_reference(name):
    m, meta, arr, x = get_model(name)
    out = m(x.to(DEV), num_registers=meta["num_registers"], return_raw_outputs=True)
    err = np.abs(out[0].float().cpu().numpy() - arr["logits"]).max()
    assert err <= FP32_TOL, f"{name}: fp32 logits max abs err {err:.3e}"
    if "raw_x" in arr:
        assert np.abs(out[1].cpu().numpy() - arr["raw_x"]).max() <= 5e-3 * max(1, np.abs(arr["raw_x"]).max())
        assert np.abs(out[2].cpu().numpy() - arr["raw_reg"]).max() <= 5e-3 * max(1, np.abs(arr["raw_reg"]).max())


@pytest.mark.parametrize("name", CASES)
def test_bf16_logits_match_reference(name):
    m, meta, arr, x = get_model(name)
    y = m(x.to(DEV).to(torch.bfloat16), num_registers=meta["num_registers"])
    assert y.dtype == torch.bfloat16
    err = np.abs(y.float().cpu().numpy() - arr["logits"]).max()
    assert err <= BF16_TOL, f"{name}: bf16 logits max abs err {err:.3e}"


@pytest.mark.parametrize("name", ["m_cf_b2", "xl_cf_b2", "xxs_cf_b4"])
def test_autocast_bf16_matches_reference(name):
    m, meta, arr, x = get_model(name)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x.to(DEV))
    assert y.dtype == torch.bfloat16
    err = np.abs(y.float().cpu().numpy() - arr["logits"]).max()
    assert err <= BF16_TOL, f"{name}: autocast bf16 err {err:.3e}"


def test_batch_invariance_full_size_bf16():
    """M at the BASELINE batch (256): every image's logits equal the same image
    run in a batch of 2 (bit-exact: all kernels are row/image independent)."""
    import model as ours
    torch.manual_seed(231424314)
    m = ours.MainModel(**synth.canonical("M")).to(DEV).eval().to(torch.bfloat16)
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(256, 3, 224, 224, generator=g).to(DEV).to(torch.bfloat16)
    y = m(x)
    assert y.shape == (256, 1000) and torch.isfinite(y.float()).all()
    for i in (0, 97, 255):
        j = 1 if i == 0 else 0
        y2 = m(torch.stack([x[i], x[j]]))
        assert torch.equal(y2[0], y[i]), f"image {i}: batch-dependent result"


def test_config4_eight_rank_shards_equal_global_batch():
    """BASELINE configs[3] (M, global batch 2048 over 8 GPUs): the shard each of the 8 ranks
    runs (sharding.shard_bounds, as bench.py assigns them) gives bit for bit the rows of the
    whole 2048-image forward, so the 8-rank job computes exactly the global batch."""
    import model as ours
    import sharding
    torch.manual_seed(231424314)
    m = ours.MainModel(**synth.canonical("M")).to(DEV).eval().to(torch.bfloat16)
    g = torch.Generator(device="cpu").manual_seed(2048)
    x = torch.randn(2048, 3, 224, 224, generator=g).to(DEV).to(torch.bfloat16)
    y = m(x)
    assert y.shape == (2048, 1000) and torch.isfinite(y.float()).all()
    for r in range(8):
        lo, hi = sharding.shard_bounds(2048, 8, r)
        assert hi - lo == 256
        assert torch.equal(m(x[lo:hi]), y[lo:hi]), f"rank {r} shard differs from the global batch"


def test_xl_full_batch_runs_finite():
    """XL at the BASELINE configs[2] batch (512): finite, and batch-invariant bit for bit."""
    import model as ours
    torch.manual_seed(1)
    m = ours.MainModel(**synth.canonical("XL")).to(DEV).eval().to(torch.bfloat16)
    x = torch.randn(512, 3, 224, 224, device=DEV, dtype=torch.bfloat16)
    y = m(x)
    assert y.shape == (512, 1000) and torch.isfinite(y.float()).all()
    y2 = m(torch.stack([x[0], x[511]]))
    assert torch.equal(y2[0], y[0]) and torch.equal(y2[1], y[511])


def _err(y, ref):
    e = float(np.abs(y - ref).max())
    return e, e / float(np.abs(ref).max())


@pytest.mark.parametrize("name", ["xxs_cf_b4", "m_cf_b2", "xl_cf_b2"])
def test_canonical_error_budget(name):
    """Per canonical size: max-abs AND max-rel-to-max|logit| error of our fp32 and bf16
    logits against the reference's fp32 CPU logits, next to the reference's OWN
    CPU-autocast-bf16 error on the same inputs (logits_autocast_bf16, generated by
    tests/golden/gen_golden.py from the reference)."""
    m, meta, arr, x = get_model(name)
    nr = meta["num_registers"]
    ref = arr["logits"]
    e32 = _err(m(x.to(DEV), num_registers=nr).float().cpu().numpy(), ref)
    e16 = _err(m(x.to(DEV).to(torch.bfloat16), num_registers=nr).float().cpu().numpy(), ref)
    eref = _err(arr["logits_autocast_bf16"], ref)
    print(f"{name}: max|logit| {np.abs(ref).max():.4f}  fp32 abs {e32[0]:.2e} rel {e32[1]:.2e}  "
          f"bf16 abs {e16[0]:.2e} rel {e16[1]:.2e}  reference-autocast abs {eref[0]:.2e} rel {eref[1]:.2e}")
    assert e32[0] <= FP32_TOL and e32[1] <= 1e-4
    assert e16[0] <= BF16_TOL and e16[1] <= 0.03
    assert e16[0] <= 4 * eref[0], "bf16 error more than 4x the reference's own autocast error"


@pytest.mark.parametrize("name", ["xxs_cf_b4", "m_cf_b2", "xl_cf_b2"])
def test_fp32_stream_eval_matches_reference_autocast(name):
    """The opt-in autocast-exact eval (model.eval_fp32_stream: the training forward's kernels with the
    residual stream in fp32, bf16 GEMM operands, dropout / drop path off) against the reference's
    fp32 logits, next to the reference's own CPU-autocast bf16 error; raw outputs too."""
    m, meta, arr, x = get_model(name)
    nr = meta["num_registers"]
    ref = arr["logits"]
    m.eval_fp32_stream = True
    try:
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(x.to(DEV), num_registers=nr)
        yb, xo, regs = m(x.to(DEV).to(torch.bfloat16), num_registers=nr, return_raw_outputs=True)
    finally:
        del m.eval_fp32_stream
    fused = _err(m(x.to(DEV).to(torch.bfloat16), num_registers=nr).float().cpu().numpy(), ref)
    e = _err(y.float().cpu().numpy(), ref)
    eb = _err(yb.float().cpu().numpy(), ref)
    eref = _err(arr["logits_autocast_bf16"], ref)
    print(f"{name}: fp32-stream eval abs {e[0]:.2e} (bf16 input {eb[0]:.2e}), fused bf16 eval {fused[0]:.2e}, "
          f"reference autocast {eref[0]:.2e}: ratios {e[0] / eref[0]:.2f} / {fused[0] / eref[0]:.2f}")
    assert y.dtype == torch.bfloat16 and yb.dtype == torch.bfloat16
    assert e[0] <= BF16_TOL and eb[0] <= BF16_TOL
    assert e[0] <= 2 * eref[0] + 1e-4, "fp32-stream eval error above twice the reference's own autocast error"
    assert xo.shape[0] == x.shape[0] and regs.shape[0] == x.shape[0]
    if "raw_x" in arr:
        assert np.abs(xo.float().cpu().numpy() - arr["raw_x"]).max() <= 2e-2 * max(1, np.abs(arr["raw_x"]).max())


def test_tanh_gelu_share_of_bf16_error():
    """The bf16 fast-GEMM epilogue uses the tanh-form GELU (declared deviation from the exact
    erf nn.GELU(), model.py:15).  Its share of the M bf16 logits error: the same forward with
    the exact-erf epilogue (sdp_gemm_set_exact_gelu) against the reference's fp32 logits."""
    import sdpnet_hip as sp
    m, meta, arr, x = get_model("m_cf_b2")
    nr = meta["num_registers"]
    ref = arr["logits"]
    xb = x.to(DEV).to(torch.bfloat16)
    e_tanh = _err(m(xb, num_registers=nr).float().cpu().numpy(), ref)
    old = sp.lib().sdp_gemm_set_exact_gelu(1)
    try:
        e_erf = _err(m(xb, num_registers=nr).float().cpu().numpy(), ref)
    finally:
        sp.lib().sdp_gemm_set_exact_gelu(old)
    print(f"m_cf_b2 bf16: tanh-form GELU abs {e_tanh[0]:.2e} rel {e_tanh[1]:.2e}; "
          f"exact-erf GELU abs {e_erf[0]:.2e} rel {e_erf[1]:.2e}")
    assert e_erf[0] <= BF16_TOL and e_tanh[0] <= BF16_TOL
    assert e_tanh[0] <= 1.5 * e_erf[0] + 2e-4, "tanh-form GELU dominates the bf16 error"


# ------------------------------------------------------------------ modules
def test_module_fixtures_on_gpu():
    z = np.load(gu.GOLDEN + "/modules.npz")
    from layers import ConvMixer, EncoderLayer, LayerNorm
    from training_utilities import KeLu
    ln = LayerNorm(48)
    ln.load_state_dict(synth.synth_state_dict(ln, 231424314))
    ln = ln.to(DEV).eval()
    y = ln(torch.from_numpy(z["cln_x"]).to(DEV))
    assert np.abs(y.cpu().numpy() - z["cln_y"]).max() <= 1e-4
    cm = ConvMixer(64, kernel_size=7, mixer_ffn_bias=True, mixer_deptwise_bias=True)
    cm.load_state_dict(synth.synth_state_dict(cm, 231424314))
    cm = cm.to(DEV).eval()
    y = cm(torch.from_numpy(z["mixer_x"]).to(DEV))
    assert np.abs(y.cpu().numpy() - z["mixer_y"]).max() <= 1e-4
    enc = EncoderLayer(64, n_head=4, activation_func=KeLu, fast_att=False)
    enc.load_state_dict(synth.synth_state_dict(enc, 231424314))
    enc = enc.to(DEV).eval()
    ye, re = enc(torch.from_numpy(z["enc_kelu_x"]).to(DEV), torch.from_numpy(z["enc_kelu_reg"]).to(DEV))
    assert np.abs(ye.cpu().numpy() - z["enc_kelu_y"]).max() <= 1e-4
    assert np.abs(re.cpu().numpy() - z["enc_kelu_yreg"]).max() <= 1e-4
    kx = torch.from_numpy(z["kelu_x"]).to(DEV)
    assert np.abs(KeLu(kx).cpu().numpy() - z["kelu_y"]).max() <= 2e-6


@pytest.mark.parametrize("conv_first", [True, False])
def test_block_and_encoder_standalone_vs_oracle(conv_first):
    from layers import Block, EncoderLayer
    import torch.nn as nn
    blk = Block(embedding_dim=96, n_head=8, conv_block_num=2, multiplication_factor=4, conv_kernel_size=7,
                conv_first=conv_first, drop_p=0.0)
    sd = synth.synth_state_dict(blk, 7)
    blk.load_state_dict(sd)
    blk = blk.to(DEV).eval()
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 96, 6, 5, generator=g)
    r = torch.randn(2, 3, 96, generator=g)
    yx, yr = blk(x.to(DEV), r.to(DEV))
    cfg = dict(orc.MAINMODEL_DEFAULTS, n_head=8, conv_first=conv_first, conv_block_num=2)
    ox, orr = orc.block(x, r, sd, "", cfg)
    assert (yx.cpu() - ox).abs().max() <= 1e-4 and (yr.cpu() - orr).abs().max() <= 1e-4
    # masked encoder, SDPA (additive float) and manual (mask==0 -> -inf) semantics
    for fast in (True, False):
        enc = EncoderLayer(96, n_head=8, fast_att=fast, activation_func=nn.GELU())
        esd = synth.synth_state_dict(enc, 8)
        enc.load_state_dict(esd)
        enc = enc.to(DEV).eval()
        N = 3 + 30
        mask = torch.ones(N, N)
        mask[:, -4:] = 0
        ex, er = enc(x.to(DEV), r.to(DEV), mask.to(DEV) if not fast else (mask > 0).to(DEV))
        rx, rr = orc.encoder_layer(x, r, esd, "", 8, "gelu", True, fast, (mask > 0) if fast else mask)
        assert (ex.cpu() - rx).abs().max() <= 1e-4 and (er.cpu() - rr).abs().max() <= 1e-4


def test_embedding_layers_and_head_standalone():
    from layers import EmbeddingLayer, ConvEmbedding, ClassificationHead, ConvPatcher
    emb = EmbeddingLayer(64, max_num_registers=5, max_image_size=[16, 16])
    sd = synth.synth_state_dict(emb, 9)
    emb.load_state_dict(sd)
    emb = emb.to(DEV)
    x = torch.randn(2, 64, 7, 9)
    xo, ro = emb(x.clone().to(DEV), 2)
    full = {"embedding_layer." + k: v for k, v in sd.items()}
    ex, er = orc.embedding_layer(x, full, 2)
    assert (xo.cpu() - ex).abs().max() <= 1e-5 and (ro.cpu() - er).abs().max() == 0
    torch.manual_seed(0)
    ce = ConvEmbedding(64, kernel_size=5, max_image_size=[16, 16], activation=torch.nn.GELU()).to(DEV)
    csd = {"embedding_layer." + k: v.cpu() for k, v in ce.state_dict().items()}
    cx, cr = ce(x.to(DEV), 3)
    ox, orr = orc.conv_embedding_layer(x, csd, 3, 5, "gelu")
    assert (cx.cpu() - ox).abs().max() <= 1e-5 and (cr.cpu() - orr).abs().max() == 0
    head = ClassificationHead(64, 10, from_register=True).eval()
    hsd = synth.synth_state_dict(head, 10)
    head.load_state_dict(hsd)
    head = head.to(DEV)
    regs = torch.randn(3, 4, 64)
    y = head(None, regs.to(DEV))
    ref = orc.classification_head(None, regs, {"output_head." + k: v for k, v in hsd.items()},
                                  dict(head_output_from_register=True, simple_mlp_output=False))
    assert (y.cpu() - ref).abs().max() <= 1e-5
    pt = ConvPatcher(64, 16)
    pt.load_state_dict(synth.synth_state_dict(pt, 11))
    pt = pt.to(DEV)
    img = torch.randn(2, 3, 64, 48)
    assert (pt(img.to(DEV)).cpu() - torch.nn.functional.conv2d(img, pt.conv.weight.cpu(), stride=16)).abs().max() <= 1e-5


def test_layer_test_hooks_fire():
    import model as ours
    torch.manual_seed(0)
    m = ours.MainModel(embedding_dim=64, num_blocks=2, n_head=4, max_image_size=[16, 16],
                       head_output_from_register=True).to(DEV)
    stats = m.layer_test()
    assert len(stats["forward_means"]) > 10 and all(np.isfinite(stats["forward_means"]))
    assert m.training  # the reference leaves the model in train mode (utility_layers.py:142)


def test_hooked_path_equals_fused_path():
    import model as ours
    meta, arr = gu.load_case("s_base")
    m, meta, arr, x = get_model("s_base")
    y_fused = m(x.to(DEV))
    h = m.blocks[0].register_forward_hook(lambda *a: None)
    try:
        y_mod = m(x.to(DEV))
    finally:
        h.remove()
    assert (y_fused - y_mod).abs().max() <= 1e-5


def test_weight_cache_invalidates_on_load_state_dict():
    m, meta, arr, x = get_model("s_base")
    y0 = m(x.to(DEV))
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    with torch.no_grad():
        m.blocks[0].t_block.ff_linear2.weight.mul_(1.5)  # (q_proj would be undone by q_norm)
    y1 = m(x.to(DEV))
    assert (y1 - y0).abs().max() > 1e-6
    m.load_state_dict(sd)
    y2 = m(x.to(DEV))
    assert torch.equal(y2, y0)


def test_cuda_graph_capture_replays_identically():
    m, meta, arr, x = get_model("xxs_cf_b4")
    xd = x.to(DEV).to(torch.bfloat16)
    mb = m
    y_eager = mb(xd)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        mb(xd)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y_static = mb(xd)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(y_static, y_eager)


def test_multistream_equals_single_stream():
    m, meta, arr, x = get_model("xxs_cf_b4")
    xd = x.to(DEV).to(torch.bfloat16).repeat(20, 1, 1, 1)[:70]
    m.num_streams = 1
    y1 = m(xd)
    m.num_streams = 3
    try:
        y3 = m(xd)
    finally:
        del m.num_streams
    torch.cuda.synchronize()
    assert torch.equal(y1, y3)


@pytest.mark.parametrize("classes,pad", [(1000, True), (1024, False)])
def test_head_padded_fast_path_matches_oracle(classes, pad):
    """ClassificationHead at batch 256 in bf16: the 1000-wide hidden layer is zero-padded to
    1024 so both head GEMMs take the MFMA fast path (layers.py ClassificationHead._prep);
    a class count that is already a multiple of 64 is not padded.  Logits vs the oracle's
    fp32 head (layers.py:449-454,462-464 of the reference)."""
    import layers
    import sdpnet_hip as sp
    torch.manual_seed(7)
    C, B, R = 768, 256, 4
    head = layers.ClassificationHead(C, classes).eval()
    with torch.no_grad():
        for prm in head.parameters():
            prm.normal_(0, 0.05)
    sd = {f"output_head.{k}": v.clone() for k, v in head.state_dict().items()}
    reg = torch.randn(B, R, C)
    head = head.to(DEV)
    w = head._prep(torch.bfloat16)["lin"]
    assert w[0][0].shape[0] == (1024 if pad else classes)
    assert sp.gemm_variant(torch.bfloat16, B, w[0][0].shape[0], C) == 1
    assert sp.gemm_variant(torch.bfloat16, B, classes, w[1][0].shape[1]) == 1
    y = head(torch.empty(0, device=DEV), reg.to(DEV).to(torch.bfloat16)).float().cpu()
    cfg = dict(head_output_from_register=True, simple_mlp_output=False)
    ref = orc.classification_head(None, reg, sd, cfg)
    assert y.shape == ref.shape == (B, classes)
    err = (y - ref).abs().max().item()
    scale = ref.abs().max().item()
    print(f"head classes={classes}: max abs err {err:.3e}, max |logit| {scale:.3e}, rel {err / scale:.3e}")
    assert err <= 2e-2 * scale
