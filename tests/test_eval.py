"""Evaluation ends of the path: on-device validation
preprocessing (sdp_val_preprocess), per-row metrics (sdp_logits_metrics) and the
checkpoint / run_test harness (eval_harness.py, the reference's model_test.py).

Parity anchors: the resize oracle (oracle/eval_oracle.py) is checked bit for bit
against Pillow itself (the library the reference's transforms call for PIL images;
Pillow 12.2.0 in this image and on the GPU box); the GPU kernel is then checked bit for
bit against Pillow on the uint8 crop.  Metrics are checked against torch's
cross_entropy / binary_cross_entropy_with_logits as the reference calls them.
"""
import os

import numpy as np
import pytest
import torch
from PIL import Image

import eval_oracle as eo

SIZES = [(375, 500), (500, 375), (320, 320), (320, 500), (500, 320), (100, 80), (1, 1), (333, 321),
         (640, 480), (2000, 1500), (224, 224), (17, 1800), (900, 12)]


def _image(rng, h, w, smooth):
    if smooth:  # natural-image-like gradients plus noise
        yy, xx = np.mgrid[0:h, 0:w]
        base = np.stack([(xx * 255 // max(w - 1, 1)), (yy * 255 // max(h - 1, 1)), ((xx + yy) * 7) % 256], -1)
        noise = rng.integers(-20, 21, (h, w, 3))
        return np.clip(base + noise, 0, 255).astype(np.uint8)
    return rng.integers(0, 256, (h, w, 3), dtype=np.uint8)


def _pil(img, size=(320, 320)):
    return np.asarray(Image.fromarray(img).resize((size[1], size[0]), Image.BICUBIC))


@pytest.mark.parametrize("smooth", [False, True])
def test_resize_oracle_bit_exact_vs_pillow(smooth):
    rng = np.random.default_rng(7 + smooth)
    for h, w in SIZES:
        img = _image(rng, h, w, smooth)
        np.testing.assert_array_equal(eo.pil_resize_u8(img, (320, 320)), _pil(img), err_msg=f"{h}x{w}")
    img = _image(rng, 300, 200, smooth)
    np.testing.assert_array_equal(eo.pil_resize_u8(img, (256, 288)), _pil(img, (256, 288)))


def test_center_crop_origin():
    assert eo.center_crop_origin((320, 320), (224, 224)) == (48, 48)
    assert eo.center_crop_origin((256, 257), (224, 224)) == (16, 16)  # round(16.5) = 16 (banker's)


def test_metric_oracle_matches_reference_losses():
    import training_utilities as tu
    g = torch.Generator().manual_seed(0)
    x = torch.randn(9, 1000, generator=g)
    y = torch.randint(0, 1000, (9,), generator=g)
    ce, bce, correct = eo.batch_metrics(x, y, 1000)
    assert abs(ce - float(torch.nn.CrossEntropyLoss()(x, y))) < 1e-6
    assert abs(bce - float(tu.BCEWithLogitsLoss(num_classes=1000, label_smoothing=0.0)(x, y))) < 1e-7
    assert correct == int((x.argmax(1) == y).sum())


def test_preprocess_weights_and_return_model(tmp_path):
    import eval_harness as eh
    import model as ours
    cfg = dict(embedding_dim=64, num_blocks=1, n_head=4, patch_size=16, conv_kernel_size=7, output_classes=10)
    torch.manual_seed(0)
    m = ours.MainModel.from_dict(**cfg)
    sd = m.state_dict()
    ddp = {"module." + k: v for k, v in sd.items()}
    comp = {"_orig_mod." + k: v * 2 if v.is_floating_point() else v for k, v in sd.items()}
    assert set(eh.preprocess_weights(ddp)) == set(sd)
    assert set(eh.preprocess_weights(comp)) == set(sd)
    torch.save({"model_state_dict": ddp, "model_config": cfg, "optimizer_state": {}, "scheduler_state": {},
                "epoch": 3}, tmp_path / "ck.pt")
    torch.save(comp, tmp_path / "ema.pt")
    model, ema = eh.return_model(str(tmp_path), "ck.pt", "ema.pt")
    assert not model.training and not ema.training
    for k, v in sd.items():
        assert torch.equal(model.state_dict()[k], v)
        want = v * 2 if v.is_floating_point() else v
        assert torch.equal(ema.state_dict()[k], want)


def test_val_transform_refuses_extreme_shapes():
    import preprocess
    t = preprocess.ValTransform(device="cpu")
    with pytest.raises(NotImplementedError, match="aspect ratio"):
        t([np.zeros((1001, 10, 3), np.uint8)])
    with pytest.raises(NotImplementedError, match="taps"):
        t([np.zeros((13000, 400, 3), np.uint8)])  # 13000 / 320 -> 165 taps
    with pytest.raises(TypeError):
        t([np.zeros((10, 10, 3), np.float32)])


# ------------------------------------------------------------------- GPU
def _batch(rng):
    imgs = [_image(rng, h, w, i % 2 == 1) for i, (h, w) in enumerate(SIZES)]
    imgs.append(np.asarray(Image.fromarray(_image(rng, 60, 90, True)).convert("L")))  # grayscale -> RGB
    return imgs


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_val_preprocess_matches_pillow(dtype):
    import preprocess
    rng = np.random.default_rng(11)
    imgs = _batch(rng)
    t = preprocess.val_transforms(dtype=dtype)
    out, u8 = t(imgs, return_u8=True)
    assert out.shape == (len(imgs), 3, 224, 224) and out.dtype == dtype
    u8 = u8.cpu().numpy()
    for b, img in enumerate(imgs):
        rgb = np.asarray(Image.fromarray(img).convert("RGB"))
        want_u8 = _pil(rgb)[48:272, 48:272]
        np.testing.assert_array_equal(u8[b], want_u8, err_msg=f"image {b} {img.shape}")
        ref, _ = eo.val_transform(rgb)
        tol = 2e-6 if dtype == torch.float32 else 1.6e-2  # fp32: x/255, (x-m)/s rounding; bf16 storage
        torch.testing.assert_close(out[b].float().cpu(), ref, rtol=0, atol=tol)


@pytest.mark.gpu
def test_val_preprocess_from_pil_images_and_empty_batch():
    import preprocess
    rng = np.random.default_rng(3)
    pil = [Image.fromarray(_image(rng, 280, 410, True)), Image.fromarray(_image(rng, 500, 333, False)).convert("RGBA")]
    out = preprocess.val_transforms()(pil)
    for b, im in enumerate(pil):
        ref, _ = eo.val_transform(np.asarray(im.convert("RGB")))
        torch.testing.assert_close(out[b].cpu(), ref, rtol=0, atol=2e-6)
    assert preprocess.val_transforms()([]).shape == (0, 3, 224, 224)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("ls", [0.0, 0.1])
def test_logits_metrics_vs_torch(dtype, ls):
    import sdpnet_hip as sp
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(5)
    B, C = 37, 1000
    x = (torch.randn(B, C, generator=g) * 4).to(dtype)
    x[3, 10] = x[3, 500] = 100.0  # tie: the first maximal index wins (torch.argmax)
    y = torch.randint(0, C, (B,), generator=g)
    y[3] = 10
    m = sp.logits_metrics(x.cuda(), y.cuda(), ls).cpu()
    xf = x.float()
    ce = F.cross_entropy(xf, y, reduction="none")
    t = F.one_hot(y, C) * (1 - ls) + ls / C
    bce = F.binary_cross_entropy_with_logits(xf, t, reduction="none").sum(1)
    torch.testing.assert_close(m[:, 0], ce, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(m[:, 1], bce, rtol=1e-5, atol=1e-3)
    assert torch.equal(m[:, 2], (xf.argmax(1) == y).float())
    bad = sp.logits_metrics(x.cuda(), torch.full((B,), C, dtype=torch.int64).cuda()).cpu()
    assert torch.isnan(bad).all()


@pytest.mark.gpu
def test_run_test_end_to_end():
    import eval_harness as eh
    import model as ours
    torch.manual_seed(0)
    m = ours.MainModel(embedding_dim=64, num_blocks=1, n_head=4, patch_size=16, conv_kernel_size=7,
                       output_classes=10, head_output_from_register=True).eval().cuda()
    rng = np.random.default_rng(9)
    data = [(Image.fromarray(_image(rng, int(h), int(w), True)), int(rng.integers(0, 10)))
            for h, w in rng.integers(200, 600, (11, 2))]
    got = eh.run_test(m, None, eh.return_dataloader(data, batch_size=4), compile_model=False, num_classes=10,
                      verbose=False)
    # oracle: Pillow-exact CPU transform -> the same model -> torch losses, per batch of 4
    ces, bces, correct, n = [], [], 0, 0
    for i in range(0, len(data), 4):
        chunk = data[i:i + 4]
        xb = torch.stack([eo.val_transform(np.asarray(im))[0] for im, _ in chunk]).cuda()
        yb = torch.tensor([lab for _, lab in chunk])
        with torch.no_grad():
            logits = m(xb).cpu()
        ce, bce, c = eo.batch_metrics(logits, yb, 10)
        ces.append(ce)
        bces.append(bce)
        correct += c
        n += len(chunk)
    assert abs(got["CrossEntropyLoss"] - np.mean(ces)) < 1e-5
    assert abs(got["BCEWithLogitsLoss"] - np.mean(bces)) < 1e-5
    assert got["Accuracy"] == correct / n
    got_c = eh.run_test(m, m, eh.return_dataloader(data, batch_size=4), compile_model=True, num_classes=10,
                        verbose=False)
    assert got_c == got
