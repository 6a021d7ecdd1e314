"""Sub-module forwards in training mode (layers.py: Block / EncoderLayer / ConvMixer / the
head / LayerNorm / ConvPatcher / the embedding layers called on their own after .train()).

With dropout and drop path at 0 the train-mode forward equals the eval forward, so the
oracle (pinned by the forward and training fixtures) is the reference for the outputs and,
through torch autograd, for every parameter and input gradient: fp32 within 1e-4 of each
tensor's max |g| (relative).  With dropout on: train output differs from eval and the
backward runs finite.  bf16 autocast: finite gradients of the right dtype and shape.
"""
import numpy as np
import pytest
import torch
import torch.nn as nn

import sdpnet_oracle as orc
import synth

DEV = "cuda"
pytestmark = pytest.mark.gpu


def _rel(a, b, floor=1e-12):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return float((a - b).abs().max()) / max(float(b.abs().max()), floor)


def _check(mod, outs, ref_outs, ref_params, prefix, inputs, ref_inputs, tol=1e-4):
    """Same random cotangent on both sides; compare outputs, parameter and input grads."""
    g = torch.Generator().manual_seed(5)
    cots = [torch.randn(o.shape, generator=g) for o in ref_outs]
    for o, r in zip(outs, ref_outs):
        assert o.shape == r.shape and _rel(o, r) <= tol, _rel(o, r)
    sum((o.float() * c.to(DEV)).sum() for o, c in zip(outs, cots)).backward()
    sum((r * c).sum() for r, c in zip(ref_outs, cots)).backward()
    # floor: 1e-3 of the largest parameter gradient, so a tensor whose exact gradient is zero
    # (k_norm.bias: a shift of every key moves all scores of a query equally) is not judged
    # on rounding noise
    fl = 1e-3 * max(float(v.grad.abs().max()) for v in ref_params.values() if v.grad is not None)
    for k, p in mod.named_parameters():
        rp = ref_params[prefix + k]
        if rp.grad is None:  # unused by the forward (e.g. the other head branch)
            continue
        assert p.grad is not None, k
        assert _rel(p.grad, rp.grad, fl) <= tol, (k, _rel(p.grad, rp.grad, fl))
    for a, b in zip(inputs, ref_inputs):
        assert a.grad is not None and _rel(a.grad, b.grad) <= tol, _rel(a.grad, b.grad)


def _leaf(t):
    return t.clone().requires_grad_(True)


def _sd(mod, seed, prefix=""):
    sd = synth.synth_state_dict(mod, seed)
    mod.load_state_dict(sd)
    return {prefix + k: v.clone().requires_grad_(v.is_floating_point()) for k, v in sd.items()}


@pytest.mark.parametrize("conv_first", [True, False])
def test_block_train_mode_matches_oracle_autograd(conv_first):
    from layers import Block
    blk = Block(embedding_dim=64, n_head=4, conv_block_num=2, multiplication_factor=4, conv_kernel_size=7,
                conv_first=conv_first, drop_p=0.0, ff_dropout=0.0, att_dropout=0.0)
    osd = _sd(blk, 7)
    blk = blk.to(DEV).train()
    g = torch.Generator().manual_seed(3)
    x, r = torch.randn(2, 64, 6, 5, generator=g), torch.randn(2, 3, 64, generator=g)
    xd, rd = _leaf(x.to(DEV)), _leaf(r.to(DEV))
    yx, yr = blk(xd, rd)
    cfg = dict(orc.MAINMODEL_DEFAULTS, n_head=4, conv_first=conv_first, conv_block_num=2)
    xc, rc = _leaf(x), _leaf(r)
    ox, orr = orc.block(xc, rc, osd, "", cfg)
    _check(blk, [yx, yr], [ox, orr], osd, "", [xd, rd], [xc, rc])


@pytest.mark.parametrize("fast", [True, False])
def test_encoder_layer_train_mode_matches_oracle_autograd(fast):
    from layers import EncoderLayer
    enc = EncoderLayer(64, n_head=4, fast_att=fast, activation_func=nn.GELU(), ff_dropout=0.0, att_dropout=0.0,
                       drop_p=0.0)
    osd = _sd(enc, 8)
    enc = enc.to(DEV).train()
    g = torch.Generator().manual_seed(4)
    x, r = torch.randn(3, 64, 4, 4, generator=g), torch.randn(3, 2, 64, generator=g)
    xd, rd = _leaf(x.to(DEV)), _leaf(r.to(DEV))
    yx, yr = enc(xd, rd)
    xc, rc = _leaf(x), _leaf(r)
    ox, orr = orc.encoder_layer(xc, rc, osd, "", 4, "gelu", True, fast)
    _check(enc, [yx, yr], [ox, orr], osd, "", [xd, rd], [xc, rc])


@pytest.mark.parametrize("fast", [True, False])
@pytest.mark.parametrize("bshape", [(3, 1), (1, 4)])
def test_encoder_layer_train_mode_with_mask_matches_oracle_autograd(fast, bshape):
    """A masked EncoderLayer in train mode (layers.py:289-298): SDPA attn_mask semantics (bool,
    True = attend) on the fast path, masked_fill(mask == 0, -inf) on the manual path, broadcast
    over batch or heads; the masked route is the materialised softmax.  Outputs and every
    parameter / input gradient against oracle autograd."""
    from layers import EncoderLayer
    enc = EncoderLayer(64, n_head=4, fast_att=fast, activation_func=nn.GELU(), ff_dropout=0.0, att_dropout=0.0,
                       drop_p=0.0)
    osd = _sd(enc, 9)
    enc = enc.to(DEV).train()
    g = torch.Generator().manual_seed(12)
    x, r = torch.randn(3, 64, 4, 4, generator=g), torch.randn(3, 2, 64, generator=g)
    N = 18
    keep = torch.rand(*bshape, N, N, generator=g) > 0.35
    keep[..., 0] = True  # every query keeps one key (a fully masked row is NaN on both sides)
    mask = keep if fast else keep.float()
    xd, rd = _leaf(x.to(DEV)), _leaf(r.to(DEV))
    yx, yr = enc(xd, rd, mask.to(DEV))
    xc, rc = _leaf(x), _leaf(r)
    ox, orr = orc.encoder_layer(xc, rc, osd, "", 4, "gelu", True, fast, mask)
    _check(enc, [yx, yr], [ox, orr], osd, "", [xd, rd], [xc, rc])


def test_masked_encoder_layer_dropout_on_attention_weights():
    """Manual path (fast_att=False) in train mode with a mask and dropout: the attention weights
    are dropped with the layer's dropout p (layers.py:297), so two seeds give different outputs,
    the same seed the same output, and the backward stays finite."""
    from layers import EncoderLayer
    enc = EncoderLayer(64, n_head=4, fast_att=False, activation_func=nn.GELU(), ff_dropout=0.3, att_dropout=0.0,
                       drop_p=0.0).to(DEV).train()
    g = torch.Generator().manual_seed(13)
    x, r = torch.randn(2, 64, 4, 4, generator=g).to(DEV), torch.randn(2, 2, 64, generator=g).to(DEV)
    mask = (torch.rand(18, 18, generator=g) > 0.3).float().to(DEV)
    mask[:, 0] = 1
    outs = []
    for seed in (1, 1, 2):
        torch.manual_seed(seed)
        xd = x.clone().requires_grad_(True)
        yx, yr = enc(xd, r, mask)
        (yx.float().square().sum() + yr.float().sum()).backward()
        assert torch.isfinite(xd.grad).all()
        assert all(torch.isfinite(p.grad).all() for p in enc.parameters() if p.grad is not None)
        outs.append(yx.detach().clone())
        enc.zero_grad(set_to_none=True)
    assert torch.equal(outs[0], outs[1]) and not torch.equal(outs[0], outs[2])


def test_conv_mixer_and_layernorm_train_mode_match_oracle_autograd():
    from layers import ConvMixer, LayerNorm
    cm = ConvMixer(64, kernel_size=5, mixer_ffn_bias=True, mixer_deptwise_bias=True, drop_p=0.0)
    osd = _sd(cm, 12)
    cm = cm.to(DEV).train()
    x = torch.randn(2, 64, 7, 6, generator=torch.Generator().manual_seed(6))
    xd, xc = _leaf(x.to(DEV)), _leaf(x)
    _check(cm, [cm(xd)], [orc.conv_mixer(xc, osd, "", "gelu")], osd, "", [xd], [xc])
    ln = LayerNorm(64)
    lsd = _sd(ln, 13)
    ln = ln.to(DEV).train()
    xd, xc = _leaf(x.to(DEV)), _leaf(x)
    _check(ln, [ln(xd)], [orc.channel_layernorm(xc, lsd["gamma"], lsd["beta"])], lsd, "", [xd], [xc])


def test_embedding_layers_patcher_and_heads_train_mode_match_oracle_autograd():
    from layers import ClassificationHead, ConvEmbedding, ConvPatcher, EmbeddingLayer
    x = torch.randn(2, 64, 7, 9, generator=torch.Generator().manual_seed(9))
    emb = EmbeddingLayer(64, max_num_registers=5, max_image_size=[16, 16], activation=nn.GELU())
    osd = _sd(emb, 9, "embedding_layer.")
    emb = emb.to(DEV).train()
    xd, xc = _leaf(x.to(DEV)), _leaf(x)
    xo, ro = emb(xd, 2)
    ex, er = orc.embedding_layer(xc, osd, 2, "gelu")
    _check(emb, [xo, ro], [ex, er], osd, "embedding_layer.", [xd], [xc])
    torch.manual_seed(0)
    ce = ConvEmbedding(64, kernel_size=5, max_image_size=[16, 16], activation=nn.GELU(), trainable_bone=True)
    csd = {"embedding_layer." + k: v.detach().clone().requires_grad_(v.is_floating_point())
           for k, v in ce.state_dict().items()}
    ce = ce.to(DEV).train()
    xd, xc = _leaf(x.to(DEV)), _leaf(x)
    cx, cr = ce(xd, 3)
    ox, orr = orc.conv_embedding_layer(xc, csd, 3, 5, "gelu")
    _check(ce, [cx, cr], [ox, orr], csd, "embedding_layer.", [xd], [xc])
    pt = ConvPatcher(64, 16)
    psd = _sd(pt, 11)
    pt = pt.to(DEV).train()
    img = torch.randn(2, 3, 70, 48, generator=torch.Generator().manual_seed(2))  # 70: 6 rows no patch covers
    imgd, imgc = _leaf(img.to(DEV)), _leaf(img)
    _check(pt, [pt(imgd)], [orc.conv_patcher(imgc, {"conv_init.conv.weight": psd["conv.weight"]})], psd, "",
           [imgd], [imgc])
    for from_reg in (True, False):
        head = ClassificationHead(64, 10, from_register=from_reg, dropout=0.0, bias=True)
        hsd = _sd(head, 10, "output_head.")
        head = head.to(DEV).train()
        regs = torch.randn(3, 4, 64, generator=torch.Generator().manual_seed(1))
        hx = torch.randn(3, 64, 5, 4, generator=torch.Generator().manual_seed(2))
        inp = _leaf(regs.to(DEV)) if from_reg else _leaf(hx.to(DEV))
        ref_in = _leaf(regs) if from_reg else _leaf(hx)
        y = head(None, inp) if from_reg else head(inp, None)
        ref = orc.classification_head(None if from_reg else ref_in, ref_in if from_reg else None, hsd,
                                      dict(head_output_from_register=from_reg, simple_mlp_output=False))
        _check(head, [y], [ref], hsd, "output_head.", [inp], [ref_in])


def test_train_mode_dropout_active_and_bf16_gradients_finite():
    from layers import Block
    torch.manual_seed(0)
    blk = Block(embedding_dim=128, n_head=4, conv_block_num=1, conv_first=True, drop_p=0.2, ff_dropout=0.2,
                att_dropout=0.2).to(DEV)
    x = torch.randn(4, 128, 8, 8, device=DEV)
    r = torch.randn(4, 3, 128, device=DEV)
    blk.eval()
    ex, er = blk(x, r)
    blk.train()
    tx, tr = blk(x, r)
    assert (tx - ex).abs().max() > 1e-3  # dropout / drop path active
    (tx.float().square().mean() + tr.float().square().mean()).backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in blk.parameters())
    blk.zero_grad(set_to_none=True)
    xd = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        bx, br = blk(xd, r)
    assert bx.dtype == torch.float32  # the fp32 residual stream, as autocast's x + branch
    (bx.square().mean() + br.square().mean()).backward()
    for p in blk.parameters():
        assert p.grad.dtype == p.dtype and p.grad.shape == p.shape and torch.isfinite(p.grad).all()
    assert torch.isfinite(xd.grad).all()
