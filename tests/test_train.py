"""Training step (BASELINE.json configs[4]): the HIP training path
against the reference's own gradients and AdamW step (tests/golden/train_*.npz, written by
tests/golden/gen_train_golden.py from /root/reference with dropout / drop path off).

CPU (always): the oracle's autograd gradients equal the fixtures (pins the oracle).
GPU: ``model.train()`` forward + our cross_entropy + backward through the HIP kernels,
fp32 (exact MFMA) and bf16 (autocast, the reference's training dtype), then our fused
AdamW (+ clip_grad_norm_) step; dropout / drop path statistics and mask consistency; a
gloo world-size-2 DDP run whose averaged gradient equals the single-process gradient.

Tolerances: fp32 gradients within 1e-4 of each tensor's max |g| (relative), loss 1e-5;
bf16 gradients (fp32 residual stream, the default) within 2x the reference's own
CPU-autocast-bf16 gradient error + 4e-2 AND within 4x that error (relative); the all-bf16
stream option within 2x + 6e-2; AdamW parameters 1e-5 absolute (fp32).
"""
import json
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import golden_util as gu
import sdpnet_oracle as orc
import synth

DEV = "cuda"
CASES = sorted(json.load(open(os.path.join(gu.GOLDEN, "TRAIN_MANIFEST.json"))))


def _case(name):
    meta, arr = gu.load_case(name)
    import model as ours
    torch.manual_seed(0)
    m = ours.MainModel.from_dict(**meta["config"])
    sd = synth.synth_state_dict(m, meta["wseed"])
    assert gu.digest(sd) == meta["weights_sha256"]
    m.load_state_dict(sd)
    x = synth.synth_images(meta["xseed"], meta["batch"], meta["image"])
    y = torch.from_numpy(arr["labels"])
    return meta, arr, m, sd, x, y


def _rel(got, ref, floor=0.0):
    """max |got - ref| over max(|ref|.max(), floor).  ``floor`` (a fraction of the largest
    gradient of the model) keeps tensors whose exact gradient is zero -- k_norm.bias: a bias
    added to every key shifts all scores of a query equally, so softmax ignores it -- from
    being judged on rounding noise."""
    return float(np.abs(got - ref).max()) / max(1e-12, float(np.abs(ref).max()), floor)


def _floor(arr):
    return 1e-3 * max(float(np.abs(v).max()) for k, v in arr.items() if k.startswith("grad/"))


@pytest.mark.parametrize("name", CASES)
def test_oracle_gradients_match_reference_fixture(name):
    meta, arr, m, sd, x, y = _case(name)
    osd = {k: v.clone().requires_grad_(v.is_floating_point()) for k, v in sd.items()}
    logits = orc.forward.__wrapped__(x, osd, meta["config"], num_registers=meta["num_registers"])
    loss = F.cross_entropy(logits, y, label_smoothing=meta["label_smoothing"])
    loss.backward()
    assert abs(float(loss) - float(arr["loss"])) <= 1e-5
    for k, _ in m.named_parameters():
        g = osd[k].grad
        assert g is not None, k
        assert _rel(g.numpy(), arr["grad/" + k], _floor(arr)) <= 1e-5, k


def _train_step(name, bf16, fp32_stream=True):
    import sdpnet_train
    sdpnet_train.set_fp32_stream(fp32_stream)
    meta, arr, m, sd, x, y = _case(name)
    m = m.to(DEV).train()
    xd, yd = x.to(DEV), y.to(DEV)
    if bf16:
        with torch.autocast("cuda", dtype=torch.bfloat16):
            logits = m(xd, num_registers=meta["num_registers"])
            loss = sdpnet_train.cross_entropy(logits, yd, meta["label_smoothing"])
    else:
        logits = m(xd, num_registers=meta["num_registers"])
        loss = sdpnet_train.cross_entropy(logits, yd, meta["label_smoothing"])
    try:
        loss.backward()
    finally:
        sdpnet_train.set_fp32_stream(True)
    return meta, arr, m, logits, loss


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("mode", ["fp32", "bf16", "bf16_stream16"])
def test_gradients_match_reference(name, mode):
    """fp32: every gradient within 1e-4 (relative) of the reference's fp32 gradient.  bf16
    (autocast, fp32 residual stream and stream gradient as autocast keeps them): each tensor's
    error within 2x the reference's OWN CPU-autocast-bf16 gradient error on the same inputs
    (grad_ac/* in the fixture) + 4e-2.  One tensor of the ReLU case, the first block's
    ff_linear1.weight, sits at 6x the CPU-autocast error (2.3e-2 vs 3.8e-3; 4.1x the same
    reference run under CUDA autocast): a ReLU mask flip at a near-zero pre-activation on this
    38-row batch.  test_bf16_gradient_error_matches_autocast_statistically shows it is a draw,
    not a bias.  bf16_stream16 (set_fp32_stream(False): the stream and its gradient stored in
    bf16) keeps the looser 2x + 6e-2 (5.6e-2 on that tensor)."""
    bf16 = mode != "fp32"
    meta, arr, m, logits, loss = _train_step(name, bf16, fp32_stream=mode != "bf16_stream16")
    assert abs(float(loss) - float(arr["loss"])) <= (2e-2 if bf16 else 1e-5), (float(loss), float(arr["loss"]))
    fl = _floor(arr)
    worst = []
    for k, p in m.named_parameters():
        assert p.grad is not None, f"{k}: no gradient"
        assert p.grad.dtype == torch.float32 and p.grad.shape == p.shape
        r = _rel(p.grad.cpu().numpy(), arr["grad/" + k], fl)
        rref = _rel(arr["grad_ac/" + k], arr["grad/" + k], fl)
        tol = {"fp32": 1e-4, "bf16": 2 * rref + 4e-2, "bf16_stream16": 2 * rref + 6e-2}[mode]
        worst.append((r / tol, r, rref, k))
    worst.sort(reverse=True)
    print(f"{name} {mode}: loss {float(loss):.6f} (ref {float(arr['loss']):.6f}); worst grads "
          + ", ".join(f"{k} {r:.2e} (reference autocast {rr:.2e})" for _, r, rr, k in worst[:4]))
    assert worst[0][0] <= 1.0, worst[:4]


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_bf16_gradient_error_matches_autocast_statistically(name):
    """Fixture weights, 8 fresh input batches: per tensor, the median over batches of (our bf16
    gradient error) / (the reference restatement's own CUDA-autocast-bf16 error), both against
    its fp32 autograd on the GPU, is <= 1.5 (measured <= 1.11 on 12 batches), and the mean
    error over the batches is <= 2x autocast's mean: our bf16 training is as accurate as
    autocast, not just within a budget.  (Single batches of the ReLU case swing either way by
    10x: a ReLU mask flip at a near-zero pre-activation moves a whole weight-gradient row.)"""
    import sdpnet_train
    meta, arr, m, sd, x0, y0 = _case(name)
    cfg = meta["config"]
    keys = [k for k, _ in m.named_parameters()]
    m = m.to(DEV).train()
    ratios = {k: [] for k in keys}
    errs = {k: [] for k in keys}
    for s_ in range(8):
        x = synth.synth_images(100 + s_, meta["batch"], meta["image"]).to(DEV)
        y = torch.randint(0, cfg["output_classes"], (meta["batch"],),
                          generator=torch.Generator().manual_seed(s_)).to(DEV)
        g = {}
        for ac in (False, True):
            osd = {k: v.to(DEV).clone().requires_grad_(v.is_floating_point()) for k, v in sd.items()}
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=ac):
                lo = F.cross_entropy(orc.forward.__wrapped__(x, osd, cfg, num_registers=meta["num_registers"]).float(),
                                     y, label_smoothing=meta["label_smoothing"])
            lo.backward()
            g[ac] = {k: osd[k].grad.float().cpu().numpy() for k in keys}
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = sdpnet_train.cross_entropy(m(x, num_registers=meta["num_registers"]), y, meta["label_smoothing"])
        loss.backward()
        fl = 1e-3 * max(float(np.abs(v).max()) for v in g[False].values())
        for k, p in m.named_parameters():
            e_ours, e_ac = _rel(p.grad.cpu().numpy(), g[False][k], fl), _rel(g[True][k], g[False][k], fl)
            ratios[k].append(e_ours / max(e_ac, 1e-9))
            errs[k].append((e_ours, e_ac))
    med = sorted(((float(np.median(v)), k) for k, v in ratios.items()), reverse=True)
    mean = sorted(((float(np.mean([a for a, _ in v]) / max(np.mean([b for _, b in v]), 1e-12)), k)
                   for k, v in errs.items()), reverse=True)
    print(f"{name}: worst median ratio to autocast", [(k, f"{a:.2f}") for a, k in med[:3]],
          "worst mean-error ratio", [(k, f"{a:.2f}") for a, k in mean[:3]])
    assert med[0][0] <= 1.5, med[:3]
    assert mean[0][0] <= 2.0, mean[:3]


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_adamw_step_matches_reference(name):
    """Our fused step (unscale 1, clip_grad_norm_(5), AdamW lr / wd of the fixture) after an fp32
    backward reproduces the reference's post-step parameters."""
    import sdpnet_train
    meta, arr, m, logits, loss = _train_step(name, False)
    opt = sdpnet_train.AdamW(m.parameters(), lr=meta["lr"], weight_decay=meta["weight_decay"])
    opt.step(grad_scale=1.0, max_norm=meta["max_norm"])
    torch.cuda.synchronize()
    for k, p in m.named_parameters():
        ref = arr["step/" + k]
        err = float(np.abs(p.detach().cpu().numpy() - ref).max())
        assert err <= 1e-5, (k, err)


@pytest.mark.gpu
def test_adamw_kernel_matches_torch_adamw_with_scaler_and_clip():
    import sdpnet_train
    torch.manual_seed(3)
    shapes = [(300, 70), (5000,), (3, 4, 5), (1,)]
    ps = [torch.randn(*s, device=DEV) for s in shapes]
    ref = [p.clone().requires_grad_(True) for p in ps]
    ours = [p.clone().requires_grad_(True) for p in ps]
    opt_r = torch.optim.AdamW(ref, lr=3e-3, weight_decay=0.05)
    opt_o = sdpnet_train.AdamW(ours, lr=3e-3, weight_decay=0.05)
    scale = 1024.0
    for it in range(3):
        gs = [torch.randn(*s, device=DEV) * (10 if it == 1 else 0.1) for s in shapes]
        for r, o, g in zip(ref, ours, gs):
            r.grad = g.clone()
            o.grad = g * scale  # scaled like scaler.scale(loss).backward()
        torch.nn.utils.clip_grad_norm_(ref, 5.0)
        opt_r.step()
        opt_o.step(grad_scale=scale, max_norm=5.0)
        for r, o in zip(ref, ours):
            assert torch.allclose(r, o, atol=2e-6, rtol=1e-5), (it, (r - o).abs().max().item())
    # a non-finite gradient skips the step and backs the scale off
    before = [o.detach().clone() for o in ours]
    ours[0].grad[0, 0] = float("inf")
    opt_o.step(grad_scale=float(opt_o.scaler[0]), max_norm=5.0)
    torch.cuda.synchronize()
    assert all(torch.equal(b, o) for b, o in zip(before, ours))
    assert float(opt_o.scaler[0]) == 65536.0 * 0.5


@pytest.mark.gpu
def test_adamw_gradient_address_table_reuse():
    """AdamW.step keeps the device table of gradient addresses while they stay put: gradients updated
    in place (same addresses, new values) and then replaced by new tensors (new addresses) both give
    torch.optim.AdamW's parameters."""
    import sdpnet_train
    torch.manual_seed(4)
    shapes = [(257, 33), (4097,), (2, 3)]
    ps = [torch.randn(*s, device=DEV) for s in shapes]
    ref = [p.clone().requires_grad_(True) for p in ps]
    ours = [p.clone().requires_grad_(True) for p in ps]
    opt_r = torch.optim.AdamW(ref, lr=2e-3, weight_decay=0.05)
    opt_o = sdpnet_train.AdamW(ours, lr=2e-3, weight_decay=0.05)
    for o, s in zip(ours, shapes):
        o.grad = torch.zeros(*s, device=DEV)
    for it in range(5):
        gs = [torch.randn(*s, device=DEV) * 0.1 for s in shapes]
        for r, o, g in zip(ref, ours, gs):
            r.grad = g.clone()
            if it < 3:
                o.grad.copy_(g)      # same addresses: the cached table
            else:
                o.grad = g.clone()   # new addresses: a new table
        opt_r.step()
        opt_o.step(grad_scale=1.0)
        for r, o in zip(ref, ours):
            assert torch.allclose(r, o, atol=2e-6, rtol=1e-5), (it, (r - o).abs().max().item())


def _torch_adamw_reference(shapes, lr=3e-3, wd=0.05, init_scale=1024.0, growth_interval=2):
    ps = [torch.randn(*sh, device=DEV) for sh in shapes]
    ref = [p.clone().requires_grad_(True) for p in ps]
    opt = torch.optim.AdamW(ref, lr=lr, weight_decay=wd)
    scaler = torch.amp.GradScaler("cuda", init_scale=init_scale, growth_interval=growth_interval)
    scaler.scale(torch.ones((), device=DEV))  # lazy-initialises the scale on the device
    return ps, ref, opt, scaler


@pytest.mark.gpu
def test_adamw_gradscaler_semantics_match_torch_step_for_step():
    """GradScaler + AdamW with an inf step in the middle (training_tools.py:91-99): the skipped step
    leaves params, moments and step counts alone, the scale backs off, the following finite steps
    use the right bias corrections, and the scale grows after `growth_interval` clean steps.
    Ours runs on the device scale (loss scaled by opt.scaler[0], grad_scale=None: no host sync)."""
    import sdpnet_train
    torch.manual_seed(5)
    shapes = [(300, 70), (5000,), (3, 4, 5), (1,)]
    ps, ref, opt_r, scaler = _torch_adamw_reference(shapes)
    ours = [p.clone().requires_grad_(True) for p in ps]
    opt_o = sdpnet_train.AdamW(ours, lr=3e-3, weight_decay=0.05, init_scale=1024.0, growth_interval=2)
    for it in range(6):
        gs = [torch.randn(*sh, device=DEV) * (8.0 if it == 3 else 0.1) for sh in shapes]
        if it in (1, 4):
            gs[1][17] = float("inf") if it == 1 else float("nan")
        s_ref = scaler.get_scale()
        for r, g in zip(ref, gs):
            r.grad = g * s_ref
        scaler.unscale_(opt_r)
        torch.nn.utils.clip_grad_norm_(ref, 5.0)
        scaler.step(opt_r)
        scaler.update()
        for o, g in zip(ours, gs):
            o.grad = opt_o.scale(g)  # grads of opt.scale(loss).backward()
        opt_o.step(grad_scale=None, max_norm=5.0)
        torch.cuda.synchronize()
        assert float(opt_o.scaler[0]) == scaler.get_scale(), it
        for r, o in zip(ref, ours):
            assert torch.allclose(r, o, atol=2e-6, rtol=1e-5), (it, (r - o).abs().max().item())
            sr, so = opt_r.state.get(r, {}), opt_o.state[o]
            if sr:
                assert float(sr["step"]) == float(so["step"]), it
                assert torch.allclose(sr["exp_avg"], so["exp_avg"], atol=1e-7, rtol=1e-5)
                assert torch.allclose(sr["exp_avg_sq"], so["exp_avg_sq"], atol=1e-9, rtol=1e-5)
    assert float(opt_o.state[ours[0]]["step"]) == 4.0  # 6 calls, 2 skipped


@pytest.mark.gpu
def test_adamw_skips_params_without_grad_and_resets_state_without_scaler_update():
    import sdpnet_train
    torch.manual_seed(6)
    shapes = [(64, 8), (33,), (7,)]
    ps, ref, opt_r, _ = _torch_adamw_reference(shapes)
    ours = [p.clone().requires_grad_(True) for p in ps]
    opt_o = sdpnet_train.AdamW(ours, lr=3e-3, weight_decay=0.05)
    for it in range(3):
        gs = [torch.randn(*sh, device=DEV) for sh in shapes]
        for r, o, g, i in zip(ref, ours, gs, range(3)):
            r.grad = None if i == 1 else g.clone()
            o.grad = None if i == 1 else g.clone()
        if it == 0:  # an inf with update_scaler=False: skipped, and the flag must not stick
            ours[0].grad[0, 0] = float("inf")
            before = [o.detach().clone() for o in ours]
            opt_o.step(grad_scale=1.0, update_scaler=False)
            torch.cuda.synchronize()
            assert all(torch.equal(b, o) for b, o in zip(before, ours))
            continue
        opt_r.step()
        opt_o.step(grad_scale=1.0, update_scaler=False)
        torch.cuda.synchronize()
        for r, o in zip(ref, ours):
            assert torch.allclose(r, o, atol=2e-6, rtol=1e-5), (it, (r - o).abs().max().item())
    assert torch.equal(ours[1], ps[1]) and not opt_o.state.get(ours[1])


@pytest.mark.gpu
def test_adamw_state_dict_reload_from_cpu_then_step():
    """Resume as training_tools.py:198 does: optimizer.load_state_dict of a CPU copy between
    steps must rebuild the device work lists (no stale pointers) and continue like torch."""
    import copy
    import sdpnet_train
    torch.manual_seed(7)
    shapes = [(100, 30), (9,)]
    ps, ref, opt_r, _ = _torch_adamw_reference(shapes)
    ours = [p.clone().requires_grad_(True) for p in ps]
    opt_o = sdpnet_train.AdamW(ours, lr=3e-3, weight_decay=0.05)
    for it in range(4):
        gs = [torch.randn(*sh, device=DEV) for sh in shapes]
        for r, o, g in zip(ref, ours, gs):
            r.grad = g.clone()
            o.grad = g.clone()
        opt_r.step()
        opt_o.step(grad_scale=1.0)
        if it == 1:
            sd = copy.deepcopy(opt_o.state_dict())
            for st in sd["state"].values():
                for k in list(st):
                    st[k] = st[k].detach().cpu().clone()
            opt_o.load_state_dict(sd)
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        torch.cuda.synchronize()
        for r, o in zip(ref, ours):
            assert torch.allclose(r, o, atol=2e-6, rtol=1e-5), (it, (r - o).abs().max().item())
    assert float(opt_o.state[ours[0]]["step"]) == 4.0


@pytest.mark.gpu
def test_dropout_and_drop_path_are_active_in_train_mode():
    """Canonical-style dropouts (0.2) and drop path: train-mode logits differ between two
    forwards and from eval; same seed -> same logits; gradients stay finite."""
    import model as ours
    import sdpnet_train
    cfg = dict(embedding_dim=64, num_blocks=2, n_head=4, conv_kernel_size=7, patch_size=16, max_image_size=[16, 16],
               head_output_from_register=True, ffn_dropout=0.2, attn_dropout=0.2, stochastic_depth_p=[0.3, 0.3],
               output_classes=10)
    torch.manual_seed(0)
    m = ours.MainModel.from_dict(**cfg).to(DEV)
    for prm in m.parameters():  # larger weights so the dropout effect is visible in the logits
        with torch.no_grad():
            prm.mul_(5)
    x = torch.randn(8, 3, 64, 64, device=DEV)
    m.train()
    torch.manual_seed(1)
    a = m(x)
    b = m(x)
    torch.manual_seed(1)
    a2 = m(x)
    assert torch.equal(a, a2)
    assert not torch.allclose(a, b)
    m.eval()
    with torch.no_grad():
        e = m(x)
    assert not torch.allclose(a, e)
    m.train()
    y = torch.randint(0, 10, (8,), device=DEV)
    loss = sdpnet_train.cross_entropy(m(x), y, 0.1)
    loss.backward()
    assert all(torch.isfinite(p.grad).all() for p in m.parameters())


@pytest.mark.gpu
def test_full_size_row_counts_against_oracle():
    """M = 32 x 196 token rows: the dW GEMMs take the split-K path and the bias sums the
    chunked reduction.  fp32 gradients of the HIP path vs autograd through the oracle."""
    import model as ours
    import sdpnet_train
    cfg = dict(embedding_dim=128, num_blocks=1, n_head=4, conv_kernel_size=7, patch_size=16, max_image_size=[16, 16],
               head_output_from_register=True, ffn_dropout=0.0, attn_dropout=0.0, output_classes=100,
               mixer_ffn_bias=True, conv_first=False)
    torch.manual_seed(0)
    m = ours.MainModel.from_dict(**cfg)
    sd = synth.synth_state_dict(m, 11)
    m.load_state_dict(sd)
    x = synth.synth_images(5, 32, 224)
    y = torch.from_numpy((synth.uniform(3, 32) * 100).astype(np.int64))
    osd = {k: v.clone().requires_grad_(v.is_floating_point()) for k, v in sd.items()}
    F.cross_entropy(orc.forward.__wrapped__(x, osd, cfg), y, label_smoothing=0.1).backward()
    m = m.to(DEV).train()
    sdpnet_train.cross_entropy(m(x.to(DEV)), y.to(DEV), 0.1).backward()
    fl = 1e-3 * max(float(osd[k].grad.abs().max()) for k, _ in m.named_parameters())
    worst = max((_rel(p.grad.cpu().numpy(), osd[k].grad.numpy(), fl), k) for k, p in m.named_parameters())
    print("full-size rows: worst fp32 grad rel err", worst)
    assert worst[0] <= 1e-4, worst


@pytest.mark.gpu
@pytest.mark.parametrize("conv_emb", [False, True])
def test_train_mode_embedding_activation_and_raw_outputs(conv_emb):
    """Train-mode surface the reference computes (layers.py:157-168 / :205, model.py:147-148):
    an embedding activation (GELU on x + pos) and return_raw_outputs=True, whose outputs carry
    gradients back into the model and into the input image (the patch conv's input gradient,
    sdp_unpatchify).  fp32 gradients vs autograd through the oracle."""
    import model as ours
    import sdpnet_train
    cfg = dict(embedding_dim=64, num_blocks=1, n_head=4, conv_kernel_size=7, patch_size=16, max_image_size=[16, 16],
               head_output_from_register=True, ffn_dropout=0.0, attn_dropout=0.0, output_classes=10,
               embedding_activation="gelu", conv_embedding=conv_emb, conv_embedding_kernel_size=5)
    torch.manual_seed(0)
    m = ours.MainModel.from_dict(**cfg)
    sd = synth.synth_state_dict(m, 31)
    m.load_state_dict(sd)
    x = synth.synth_images(6, 3, 224)
    y = torch.tensor([1, 7, 3])

    def objective(logits, xo, regs):  # a loss that reaches all three outputs
        return F.cross_entropy(logits, y.to(logits.device), label_smoothing=0.1) + (xo.float() ** 2).mean() \
            + 0.5 * regs.float().abs().mean()

    osd = {k: v.clone().requires_grad_(v.is_floating_point()) for k, v in sd.items()}
    xr = x.clone().requires_grad_(True)
    lo, xo, ro = orc.forward.__wrapped__(xr, osd, cfg, return_raw_outputs=True)
    objective(lo, xo, ro).backward()
    m = m.to(DEV).train()
    xd = x.to(DEV).requires_grad_(True)
    lg, xg, rg = m(xd, return_raw_outputs=True)
    assert xg.shape == xo.shape and rg.shape == ro.shape
    assert float((xg.cpu() - xo.detach()).abs().max()) <= 1e-4
    objective(lg, xg, rg).backward()
    fl = 1e-3 * max(float(osd[k].grad.abs().max()) for k, _ in m.named_parameters())
    worst = max((_rel(p.grad.cpu().numpy(), osd[k].grad.numpy(), fl), k) for k, p in m.named_parameters())
    assert worst[0] <= 1e-4, worst
    assert xd.grad is not None and xd.grad.shape == xr.grad.shape
    assert _rel(xd.grad.cpu().numpy(), xr.grad.numpy(), 1e-3 * float(xr.grad.abs().max())) <= 1e-4


XL_TRAIN_CFG = dict(embedding_dim=768, num_blocks=2, n_head=8, conv_kernel_size=7, patch_size=14,
                    max_image_size=[16, 16], max_num_registers=5, head_output_from_register=True, conv_first=True,
                    normalize_qv=True, ffn_dropout=0.0, attn_dropout=0.0, stochastic_depth_p=[0.0, 0.0],
                    output_classes=1000, activation="gelu")


@pytest.mark.gpu
def test_xl_architecture_training_step_against_oracle():
    """BASELINE.json configs[4]'s architecture (training_tools.py:77-103): SdP-Net-XL's block
    dimensions -- d 768, 8 heads of 96, patch 14, 256 patches + 4 registers = 260 tokens -- with
    2 blocks to keep the CPU side cheap, batch 2.  fp32: every HIP gradient within 1e-4 (relative)
    of autograd through the oracle (pinned by the train fixtures); the fused AdamW step equals
    torch.optim.AdamW + clip_grad_norm_ on the same gradients.  bf16 (autocast, fp32 residual
    stream): each gradient's error within min(2x the oracle's own CPU-autocast error + 4e-2, 4x
    that error) (the fixture rule)."""
    import model as ours
    import sdpnet_train
    cfg = XL_TRAIN_CFG
    torch.manual_seed(0)
    m = ours.MainModel.from_dict(**cfg)
    sd = synth.synth_state_dict(m, 21)
    m.load_state_dict(sd)
    x = synth.synth_images(9, 2, 224)
    y = torch.tensor([3, 917])
    osd = {k: v.clone().requires_grad_(v.is_floating_point()) for k, v in sd.items()}
    F.cross_entropy(orc.forward.__wrapped__(x, osd, cfg), y, label_smoothing=0.1).backward()
    ref = {k: osd[k].grad.numpy() for k, _ in m.named_parameters()}
    asd = {k: v.clone().requires_grad_(v.is_floating_point()) for k, v in sd.items()}
    with torch.autocast("cpu", dtype=torch.bfloat16):
        lac = F.cross_entropy(orc.forward.__wrapped__(x, asd, cfg), y, label_smoothing=0.1)
    lac.backward()
    fl = 1e-3 * max(float(np.abs(g).max()) for g in ref.values())
    m = m.to(DEV).train()
    for bf16 in (False, True):
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
            loss = sdpnet_train.cross_entropy(m(x.to(DEV)), y.to(DEV), 0.1)
        loss.backward()
        worst = []
        for k, p in m.named_parameters():
            r = _rel(p.grad.cpu().numpy(), ref[k], fl)
            rac = _rel(asd[k].grad.float().numpy(), ref[k], fl)
            tol = min(2 * rac + 4e-2, 4 * rac) if bf16 else 1e-4
            worst.append((r / tol, r, rac, k))
        worst.sort(reverse=True)
        print(f"XL-dim training bf16={bf16}: worst", [(k, f"{r:.2e}", f"{rac:.2e}") for _, r, rac, k in worst[:3]])
        assert worst[0][0] <= 1.0, worst[:3]
    # fused AdamW (+ clip) vs torch.optim.AdamW on the same (bf16-path) gradients
    params = [p for p in m.parameters()]
    ref_p = [p.detach().clone().requires_grad_(True) for p in params]
    for rp, p in zip(ref_p, params):
        rp.grad = p.grad.detach().clone()
    torch.nn.utils.clip_grad_norm_(ref_p, 5.0)
    torch.optim.AdamW(ref_p, lr=0.0015, weight_decay=0.05).step()
    sdpnet_train.AdamW(params, lr=0.0015, weight_decay=0.05).step(grad_scale=1.0, max_norm=5.0)
    torch.cuda.synchronize()
    err = max(float((rp - p).abs().max()) for rp, p in zip(ref_p, params))
    assert err <= 1e-5, err


@pytest.mark.gpu
def test_xl_full_size_training_step_is_deterministic():
    """The benchmarked XL training step at its full per-GPU batch (120 images, configs[4]):
    two runs from the same seeds give bit-identical parameters after one fused step (dropout
    masks from the counter hash, split-K reductions and the gradient norm in a fixed order),
    and every gradient is finite."""
    import model as ours
    import sdpnet_train
    cfg = dict(XL_TRAIN_CFG, num_blocks=17, ffn_dropout=0.2, attn_dropout=0.2)
    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randn(120, 3, 224, 224, generator=g).to(DEV)
    y = torch.randint(0, 1000, (120,), generator=g).to(DEV)
    outs = []
    for _ in range(2):
        torch.manual_seed(231424314)
        m = ours.MainModel.from_dict(**cfg).to(DEV).train()
        opt = sdpnet_train.AdamW(m.parameters(), lr=0.0015, weight_decay=0.05)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = sdpnet_train.cross_entropy(m(x), y, 0.1)
        opt.scale(loss).backward()
        assert all(torch.isfinite(p.grad).all() for p in m.parameters())
        opt.step(grad_scale=None, max_norm=5.0)
        torch.cuda.synchronize()
        assert float(opt._steps[0]) == 1.0  # the step was taken (no inf / nan)
        outs.append(torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu())
        del m, opt
        torch.cuda.empty_cache()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.gpu
def test_batched_weight_prep_is_bit_identical_over_two_steps():
    """The per-step bf16 weight operands (and their transposes for the input-gradient GEMMs)
    built in one sdp_mt_cast_transpose launch give the same bits as the per-weight cast /
    transpose path, over two AdamW steps (the second forward must see the updated weights)."""
    import model as ours
    import sdpnet_train
    cfg = dict(XL_TRAIN_CFG, num_blocks=2, ffn_dropout=0.2, attn_dropout=0.2)
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randn(4, 3, 224, 224, generator=g).to(DEV)
    y = torch.randint(0, 1000, (4,), generator=g).to(DEV)
    res = {}
    old = sdpnet_train._WPREP_ON
    try:
        for on in (True, False):
            sdpnet_train._WPREP_ON = on
            torch.manual_seed(231424314)
            m = ours.MainModel.from_dict(**cfg).to(DEV).train()
            opt = sdpnet_train.AdamW(m.parameters(), lr=0.01, weight_decay=0.05)
            grads = []
            for step in range(2):
                torch.manual_seed(100 + step)
                m.zero_grad(set_to_none=True)
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    loss = sdpnet_train.cross_entropy(m(x), y, 0.1)
                loss.backward()
                grads.append(torch.cat([p.grad.reshape(-1) for p in m.parameters()]).cpu())
                opt.step(grad_scale=1.0, max_norm=5.0)
            torch.cuda.synchronize()
            res[on] = grads
            assert on == ("_sdp_wprep" in m.__dict__)
    finally:
        sdpnet_train._WPREP_ON = old
    for a, b in zip(res[True], res[False]):
        assert torch.equal(a, b)


@pytest.mark.gpu
def test_side_stream_weight_gradients_are_bit_identical():
    """The layers' weight gradients computed on the side stream (overlapping the dX chain) equal
    the single-stream ones bit for bit, and the step after them sees finished gradients."""
    import model as ours
    import sdpnet_train
    cfg = dict(XL_TRAIN_CFG, num_blocks=2, ffn_dropout=0.2, attn_dropout=0.2)
    g = torch.Generator(device="cpu").manual_seed(6)
    x = torch.randn(4, 3, 224, 224, generator=g).to(DEV)
    y = torch.randint(0, 1000, (4,), generator=g).to(DEV)
    res = {}
    old = sdpnet_train._WSTREAM
    try:
        for on in (True, False):
            sdpnet_train._WSTREAM = on
            torch.manual_seed(231424314)
            m = ours.MainModel.from_dict(**cfg).to(DEV).train()
            opt = sdpnet_train.AdamW(m.parameters(), lr=0.01, weight_decay=0.05)
            out = []
            for step in range(2):
                torch.manual_seed(200 + step)
                m.zero_grad(set_to_none=True)
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    loss = sdpnet_train.cross_entropy(m(x), y, 0.1)
                loss.backward()
                out.append(torch.cat([p.grad.reshape(-1) for p in m.parameters()]).cpu())
                opt.step(grad_scale=1.0, max_norm=5.0)
            out.append(torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu())
            res[on] = out
    finally:
        sdpnet_train._WSTREAM = old
    for a, b in zip(res[True], res[False]):
        assert torch.equal(a, b)


def test_mt_cast_transpose_entry_layout():
    import sdpnet_hip as sp
    assert sp.lib().sdp_mt_cast_transpose_entry_bytes() == 48


class _OracleModule(torch.nn.Module):
    """The oracle forward (reference math, stock torch CPU ops) as a module whose parameters
    DDP can hook (CPU gloo test of the data-parallel gradient average)."""

    def __init__(self, sd, cfg, nreg):
        super().__init__()
        self.names = [k for k, v in sd.items() if v.is_floating_point()]
        self.params = torch.nn.ParameterList([torch.nn.Parameter(sd[k].clone()) for k in self.names])
        self.bufs = {k: v for k, v in sd.items() if not v.is_floating_point()}
        self.cfg, self.nreg = cfg, nreg

    def forward(self, x):
        sd = dict(self.bufs)
        sd.update(zip(self.names, self.params))
        return orc.forward.__wrapped__(x, sd, self.cfg, num_registers=self.nreg)


def _ddp_worker(rank, world, port, q, gpu):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        name = CASES[0]
        meta, arr, m, sd, x, y = _case(name)
        B = x.shape[0]
        lo, hi = (0, 2) if rank == 0 else (2, B)
        if gpu:  # our HIP training path, both ranks on the one GPU of the box
            import sdpnet_train
            m = m.to(DEV).train()
            ddp = torch.nn.parallel.DistributedDataParallel(m)
            logits = ddp(x[lo:hi].to(DEV), num_registers=meta["num_registers"])
            yy = y[lo:hi].to(DEV)
            # DDP averages over ranks: scale the local mean so the average is the global mean
            loss = sdpnet_train.cross_entropy(logits, yy, meta["label_smoothing"]) * ((hi - lo) * world / B)
            named = dict(m.named_parameters())
        else:
            om = _OracleModule(sd, meta["config"], meta["num_registers"])
            ddp = torch.nn.parallel.DistributedDataParallel(om)
            logits = ddp(x[lo:hi])
            loss = F.cross_entropy(logits, y[lo:hi], label_smoothing=meta["label_smoothing"]) * ((hi - lo) * world / B)
            named = dict(zip(om.names, om.params))
        loss.backward()  # DDP's bucketed all-reduce (mean) runs in the backward hooks
        if rank == 0:
            q.put({k: p.grad.detach().cpu().numpy().copy() for k, p in named.items()})
    finally:
        dist.destroy_process_group()


def _run_two_ranks(gpu):
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q, gpu)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        grads = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    _, arr = gu.load_case(CASES[0])
    worst = max(_rel(g, arr["grad/" + k], _floor(arr)) for k, g in grads.items())
    return worst


def test_two_rank_ddp_gradient_average_matches_single_process():
    """World-size-2 gloo DDP over the oracle module: each rank's shard gradient, averaged by
    DDP's all-reduce, equals the reference's full-batch gradient (fixture)."""
    assert _run_two_ranks(False) <= 1e-5


@pytest.mark.gpu
def test_two_rank_ddp_on_hip_training_path():
    """The same through DDP(MainModel) on the HIP training path (two gloo ranks sharing the
    box's GPU; RCCL needs one GPU per rank, the bench's 8-GPU run uses it)."""
    assert _run_two_ranks(True) <= 1e-4
