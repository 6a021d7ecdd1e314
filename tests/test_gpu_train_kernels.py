"""GPU: the training-step kernels (csrc/train.hip) against plain PyTorch fp32 references of the
same ops (torch autograd for the backward ones).  Tolerances: fp32 paths ~1e-5 relative to
the reference's max magnitude; bf16 operands 2e-2."""
import math

import pytest
import torch
import torch.nn.functional as F

import sdpnet_hip as sp

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def rnd(*shape, seed=0, dtype=torch.float32, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dtype).to(DEV)


def close(got, ref, rel, what=""):
    got, ref = got.float(), ref.float()
    err = (got - ref).abs().max().item()
    scale = max(1.0, ref.abs().max().item()) if rel >= 1e-3 else max(1e-6, ref.abs().max().item())
    assert err <= rel * scale, f"{what}: max abs err {err:.3e} vs scale {scale:.3e} (rel tol {rel})"


def _logical(t, trans):
    return t.t() if trans else t


@pytest.mark.parametrize("dtype", [torch.float32, BF])
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(128, 128, 32), (260, 96, 260), (200, 768, 96), (77, 300, 1000), (1, 17, 8)])
def test_gemm_flex(dtype, ta, tb, M, N, K):
    # bf16 rows must be 16-B aligned: pad the stored row length to a multiple of 8
    def padded(r, c, seed):
        cp = (c + 7) // 8 * 8
        return rnd(r, cp, seed=seed, dtype=dtype)[:, :c]
    A = padded(*((K, M) if ta else (M, K)), 1)
    B = padded(*((N, K) if tb else (K, N)), 2)
    C = torch.empty(M, N, dtype=torch.float32, device=DEV)
    sp.gemm_flex(A, B, C, M, N, K, ta=ta, tb=tb, alpha=0.5, lda=A.stride(0), ldb=B.stride(0))
    ref = 0.5 * _logical(A.float(), ta) @ _logical(B.float(), tb)
    close(C, ref, 1e-5 if dtype == torch.float32 else 2e-2, f"flex ta={ta} tb={tb}")


@pytest.mark.parametrize("ta,tb", [(0, 1), (1, 0)])
def test_gemm_flex_bf16_out_accum_and_batched(ta, tb):
    # batched over (b, h) with two-level strides, as the attention products use it
    Bn, H, Nq, d = 3, 4, 70, 32
    q = rnd(Bn, Nq, 3 * H * d, seed=3, dtype=BF)
    out = torch.zeros(Bn, H, Nq, Nq if tb else d, dtype=BF, device=DEV)
    if tb:  # S = Q K^T per (b, h)
        sp.gemm_flex(q, q, out, Nq, Nq, d, ta=False, tb=True, lda=3 * H * d, ldb=3 * H * d, ldc=Nq, Z=Bn * H, zdiv=H,
                     sa=(Nq * 3 * H * d, d), sb=(Nq * 3 * H * d, d), sc=(H * Nq * Nq, Nq * Nq), b_off=H * d)
        qq = q.float().view(Bn, Nq, 3, H, d)
        ref = torch.einsum("bqhd,bkhd->bhqk", qq[:, :, 0], qq[:, :, 1])
    else:  # dK = P^T Q per (b, h) with P [Nq, Nq]
        P = rnd(Bn, H, Nq, 72, seed=4, dtype=BF)[..., :Nq]  # rows padded to 16 B
        sp.gemm_flex(P, q, out, Nq, d, Nq, ta=True, tb=False, lda=72, ldb=3 * H * d, ldc=d, Z=Bn * H, zdiv=H,
                     sa=(H * Nq * 72, Nq * 72), sb=(Nq * 3 * H * d, d), sc=(H * Nq * d, Nq * d))
        qq = q.float().view(Bn, Nq, 3, H, d)
        ref = torch.einsum("bhkq,bkhd->bhqd", P.float(), qq[:, :, 0])
    close(out, ref, 2e-2, "batched flex")
    # accumulate into fp32
    A = rnd(64, 96, seed=5, dtype=BF)
    Bm = rnd(40, 96, seed=6, dtype=BF)
    C = rnd(64, 40, seed=7)
    C0 = C.clone()
    sp.gemm_flex(A, Bm, C, 64, 40, 96, tb=True, accum=True)
    close(C, C0 + A.float() @ Bm.float().t(), 2e-2, "accum")


@pytest.mark.parametrize("dtype", [torch.float32, BF])
def test_gemm_flex_split_k_dW(dtype):
    """dW = dY^T X (both operands token-major) with split-K slabs reduced by seg_colsum."""
    M, N, K, S = 3000, 192, 256, 5
    dy = rnd(M, N, seed=8, dtype=dtype)
    x = rnd(M, K, seed=9, dtype=dtype)
    slabs = torch.empty(S, N, K, dtype=torch.float32, device=DEV)
    sp.gemm_flex(dy, x, slabs, N, K, M, ta=True, tb=False, splits=S, split_stride=N * K)
    dw = torch.empty(N, K, dtype=torch.float32, device=DEV)
    sp.seg_colsum(slabs.view(S, N * K), dw.view(1, N * K), 1, S, 0, 1, N * K)
    close(dw, dy.float().t() @ x.float(), 1e-5 if dtype == torch.float32 else 2e-2, "split-K dW")


@pytest.mark.parametrize("dtype", [torch.float32, BF])
def test_seg_colsum(dtype):
    X = rnd(6 * 50, 70, seed=10, dtype=dtype)
    out = torch.empty(6, 70, dtype=torch.float32, device=DEV)
    sp.seg_colsum(X, out, 6, 50, 1, 6, 70)  # group g = rows g, g+6, g+12, ...
    close(out, X.float().view(50, 6, 70).sum(0), 1e-5, "strided segments")
    out2 = torch.ones(1, 70, device=DEV)
    sp.seg_colsum(X, out2, 1, 300, 0, 1, 70, scale=0.5, accum=True)
    close(out2, 1 + 0.5 * X.float().sum(0, keepdim=True), 1e-5, "scaled accumulate")


@pytest.mark.parametrize("dtype", [torch.float32, BF])
@pytest.mark.parametrize("G,len_,C", [(3, 77, 1024), (1, 28, 4096), (1, 7, 2048), (122, 256, 768), (1, 122, 3072)])
def test_seg_colsum_vec4_summation_order(dtype, G, len_, C):
    # the 4-column kernel (C % 4 == 0): thread slice sl sums rows sl, sl + 4, ... in row order,
    # slices combined as ((s0 + s1) + s2) + s3 -- reproduced exactly in fp32 on the host
    X = rnd(G * len_, C, seed=11, dtype=dtype)
    out = torch.empty(G, C, dtype=torch.float32, device=DEV)
    sp.seg_colsum(X, out, G, len_, len_, 1, C)
    Xh = X.float().cpu().view(G, len_, C)
    sl = []
    for k in range(4):
        acc = torch.zeros(G, C, dtype=torch.float32)
        for e in range(k, len_, 4):
            acc = acc + Xh[:, e]
        sl.append(acc)
    ref = ((sl[0] + sl[1]) + sl[2]) + sl[3]
    assert torch.equal(out.cpu(), ref)


@pytest.mark.parametrize("len_,C", [(7, 768 * 3072), (28, 768 * 768), (9, 2304 * 768), (3, 65536), (64, 131072)])
def test_seg_colsum_wide_slab_sum_in_row_order(len_, C):
    # the weight-gradient slab reduction (G = 1, few rows, C = N x K): out = ((x0 + x1) + x2) + ...
    X = rnd(len_, C, seed=12)
    out = torch.empty(1, C, dtype=torch.float32, device=DEV)
    sp.seg_colsum(X, out, 1, len_, 0, 1, C)
    Xh = X.cpu()
    ref = torch.zeros(C, dtype=torch.float32)
    for e in range(len_):
        ref = ref + Xh[e]
    assert torch.equal(out.cpu()[0], ref)
    out2 = torch.ones(1, C, device=DEV)
    sp.seg_colsum(X, out2, 1, len_, 0, 1, C, scale=0.5, accum=True)
    assert torch.equal(out2.cpu()[0], 1 + 0.5 * ref)


ACT_REF = {0: lambda x: x, 1: F.gelu, 2: F.relu, 3: torch.tanh, 4: torch.sigmoid,
           5: lambda x: F.leaky_relu(x, 0.01), 6: F.selu,
           7: lambda x: torch.where(x < -3.5, torch.zeros_like(x), torch.where(
               x > 3.5, x, 0.5 * x * (1 + x / 3.5 + torch.sin(math.pi * x / 3.5) / math.pi)))}


@pytest.mark.parametrize("code", list(ACT_REF))
@pytest.mark.parametrize("dtype", [torch.float32, BF])
def test_act_fwd_bwd(code, dtype):
    M, N = 33, 257
    z = (torch.linspace(-6, 6, M * N, device=DEV).view(M, N) + 0.013).to(dtype)
    dy = rnd(M, N, seed=11, dtype=dtype)
    y = torch.empty_like(z)
    dz = torch.empty_like(z)
    sp.act_fwd(z, y, M, N, code)
    sp.act_bwd(z, dy, dz, M, N, code)
    zr = z.float().clone().requires_grad_(True)
    yr = ACT_REF[code](zr)
    (gz,) = torch.autograd.grad(yr, zr, dy.float())
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    close(y, yr.detach(), tol, f"act {code} fwd")
    close(dz, gz, tol, f"act {code} bwd")


def test_dropout_mask_consistent():
    M, N, p = 512, 1024, 0.2
    z = rnd(M, N, seed=12).abs() + 0.5  # no exact zeros: y != 0 is the keep mask
    y = torch.empty_like(z)
    sp.act_fwd(z, y, M, N, 0, p=p, seed=1234)
    keep = y != 0
    rate = keep.float().mean().item()
    assert abs(rate - (1 - p)) < 0.005, rate
    close(y[keep], z[keep] / (1 - p), 1e-6, "kept values scaled")
    dz = torch.empty_like(z)
    ones = torch.ones_like(z)
    sp.act_bwd(z, ones, dz, M, N, 0, p=p, seed=1234)
    bad = ((dz != 0) != keep).sum().item()
    assert bad == 0, (bad, dz[(dz != 0) != keep][:8].tolist(), z[(dz != 0) != keep][:8].tolist())
    y2 = torch.empty_like(z)
    sp.act_fwd(z, y2, M, N, 0, p=p, seed=1235)
    assert not torch.equal(y2 != 0, keep)


@pytest.mark.parametrize("p", [0.0, 0.3])
@pytest.mark.parametrize("code", [0, 1, 2])
def test_act_vector_path_equals_elementwise_path(code, p):
    """The 8-wide act kernels (compile-time activation, 32-bit items, split dropout hash) against the
    one-element kernels (uniform01 per element): an odd row stride sends the same rows (same
    dropout indices m * N + n) down the second path."""
    M, N = 77, 1024
    zs = rnd(M, N + 1, seed=41, dtype=BF)
    dys = rnd(M, N + 1, seed=42, dtype=BF)
    z, dy = zs[:, :N].contiguous(), dys[:, :N].contiguous()
    yv, ye = torch.empty(M, N, device=DEV, dtype=BF), torch.zeros(M, N + 1, device=DEV, dtype=BF)
    sp.act_fwd(z, yv, M, N, code, p=p, seed=99)
    sp.act_fwd(zs, ye, M, N, code, p=p, seed=99, ldz=N + 1, ldy=N + 1)
    assert torch.equal(yv, ye[:, :N])
    dv, de = torch.empty(M, N, device=DEV, dtype=BF), torch.zeros(M, N + 1, device=DEV, dtype=BF)
    sp.act_bwd(z, dy, dv, M, N, code, p=p, seed=99)
    sp.act_bwd(zs, dys, de, M, N, code, p=p, seed=99, ld=N + 1)
    assert torch.equal(dv, de[:, :N])


@pytest.mark.parametrize("dtype", [torch.float32, BF])
@pytest.mark.parametrize("M,C,eps", [(300, 768, 1e-6), (77, 96, 1e-5), (5, 64, 1e-5), (20011, 96, 1e-5),
                                     (333, 128, 1e-5), (70, 32, 1e-5)])
def test_layernorm_fwd_bwd(dtype, M, C, eps):
    x = (rnd(M, C, seed=13, scale=1.5) + rnd(M, 1, seed=14, scale=2)).to(dtype)
    g = rnd(C, seed=15) * 0.2 + 1
    b = rnd(C, seed=16) * 0.2
    dy = rnd(M, C, seed=17, dtype=dtype)
    add = rnd(M, C, seed=18, dtype=dtype)
    st = torch.empty(M, 2, device=DEV)
    sp.rowstats(sp.dense(x), eps, st, M, C)
    y = torch.empty_like(x)
    sp.ln_apply(sp.dense(x), st, g, b, sp.dense(y), M, C)
    dx = torch.empty_like(x)
    dg, db = sp.ln_bwd(sp.dense(x), st, g, sp.dense(dy), sp.dense(dx), M, C, add=sp.dense(add))
    xr = x.float().clone().requires_grad_(True)
    gr, br = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = F.layer_norm(xr, (C,), gr, br, eps)
    gx, gg, gb = torch.autograd.grad(yr, (xr, gr, br), dy.float())
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    close(y, yr.detach(), tol, "ln fwd")
    close(dx, gx + add.float(), tol * 4, "ln dx")
    close(dg, gg, tol * 4, "ln dgamma")
    close(db, gb, tol * 4, "ln dbeta")


@pytest.mark.parametrize("dtype", [torch.float32, BF])
def test_softmax_fwd_bwd(dtype):
    rows, N, Npad, scale = 96, 260, 264, 1 / math.sqrt(96)
    S = rnd(rows, Npad, seed=19, scale=4)
    P = torch.empty(rows, Npad, dtype=dtype, device=DEV)
    sp.softmax_fwd(S, P, None, rows, N, Npad, scale)
    Sr = S[:, :N].clone().requires_grad_(True)
    Pr = torch.softmax(Sr * scale, -1)
    tol = 2e-6 if dtype == torch.float32 else 1e-2
    close(P[:, :N], Pr.detach(), tol, "softmax")
    assert (P[:, N:] == 0).all()
    dP = rnd(rows, Npad, seed=20, dtype=dtype)
    dS = torch.empty(rows, Npad, dtype=dtype, device=DEV)
    sp.softmax_bwd(P, dP, dS, rows, N, Npad)
    (gS,) = torch.autograd.grad(Pr, Sr, dP[:, :N].float())
    close(dS[:, :N] * scale, gS, 1e-5 if dtype == torch.float32 else 2e-2, "softmax bwd")


def test_softmax_dropout_mask_consistent():
    rows, N, p = 64, 200, 0.2
    S = rnd(rows, N, seed=21)
    P = torch.empty(rows, N, device=DEV)
    Pd = torch.empty(rows, N, device=DEV)
    sp.softmax_fwd(S, P, Pd, rows, N, N, 1.0, p=p, seed=77)
    keep = Pd != 0
    close(Pd[keep], P[keep] / (1 - p), 1e-6, "dropped softmax scaled")
    dS = torch.empty_like(P)
    sp.softmax_bwd(P, torch.ones_like(P), dS, rows, N, N, p=p, seed=77)
    Pr = torch.softmax(S.clone().requires_grad_(True), -1)
    mask = keep.float() / (1 - p)
    ref = P * (mask - (mask * P).sum(-1, keepdim=True))
    close(dS, ref, 1e-5, "dropout softmax bwd")


@pytest.mark.parametrize("dtype", [torch.float32, BF])
@pytest.mark.parametrize("B,H,W,C,k", [(3, 14, 14, 128, 7), (2, 16, 16, 64, 3), (2, 7, 9, 96, 5), (3, 12, 24, 72, 7),
                                     (130, 16, 16, 96, 7), (2, 20, 24, 40, 7)])
def test_dw_wgrad(dtype, B, H, W, C, k):
    a = rnd(B * H * W, C, seed=22, dtype=dtype)
    dy = rnd(B * H * W, C, seed=23, dtype=dtype)
    got = sp.dw_wgrad(sp.dense(a), sp.dense(dy), B, H, W, C, k)
    an = a.float().view(B, H, W, C).permute(0, 3, 1, 2)
    w = torch.zeros(C, 1, k, k, device=DEV, requires_grad=True)
    y = F.conv2d(an, w, padding="same", groups=C)
    (gw,) = torch.autograd.grad(y, w, dy.float().view(B, H, W, C).permute(0, 3, 1, 2))
    close(got, gw.view(C, k * k), 1e-4 if dtype == torch.float32 else 2e-2, "dw wgrad")


@pytest.mark.parametrize("N,K,M,kchunk", [(256, 256, 64, 1), (256, 512, 640, 3), (768, 768, 30720, 18),
                                          (512, 256, 4096, 64), (2304, 768, 1024, 4), (256, 256, 37, 1),
                                          (768, 512, 31200, 55), (256, 768, 700, 4)])
def test_gemm_wgrad_8ph(N, K, M, kchunk):
    # dW = dY^T X on the 8-phase kernel (csrc/wgrad.hip) vs fp32 torch; each split's slab alone
    # too; M % 64 != 0: the last K-tile reads the zero row past the last token
    dy = rnd(M, N, seed=31, dtype=BF, scale=0.5)
    x = rnd(M, K, seed=32, dtype=BF)
    nkt = -(-M // 64)
    splits = -(-nkt // kchunk)
    slabs = torch.full((splits, N, K), float("nan"), device=DEV)
    sp.gemm_wgrad(dy, x, slabs, M, kchunk, split_stride=N * K)
    for s in range(splits):
        lo, hi = s * kchunk * 64, min(M, (s + 1) * kchunk * 64)
        ref = dy[lo:hi].float().t() @ x[lo:hi].float()
        close(slabs[s], ref, 1e-5, f"wgrad slab {s}")
    close(slabs.sum(0), dy.float().t() @ x.float(), 1e-5, "wgrad sum")


@pytest.mark.parametrize("N,K,M,kchunk", [(256, 256, 64, 1), (256, 512, 640, 3), (768, 768, 30720, 18),
                                          (256, 256, 37, 1), (768, 512, 4136, 5)])
def test_gemm_wgrad_kloop_phases_bit_identical(N, K, M, kchunk):
    # the 2-phase main loop (default) accumulates in the 4-phase loop's order: identical slabs
    dy = rnd(M, N, seed=35, dtype=BF, scale=0.5)
    x = rnd(M, K, seed=36, dtype=BF)
    splits = -(-(-(-M // 64)) // kchunk)
    outs = []
    diag = sp.lib().sdp_build_info() != 0  # the 4-phase loop exists only in the diagnostic build
    for ph in ((4, 2) if diag else (2,)):
        old = sp.lib().sdp_gemm_set_kloop_phases(ph)
        assert old >= 0
        try:
            slabs = torch.full((splits, N, K), float("nan"), device=DEV)
            sp.gemm_wgrad(dy, x, slabs, M, kchunk, split_stride=N * K)
            torch.cuda.synchronize()
            outs.append(slabs)
        finally:
            sp.lib().sdp_gemm_set_kloop_phases(old)
    if len(outs) == 2:
        assert torch.equal(outs[0], outs[1])
    close(outs[-1].sum(0), dy.float().t() @ x.float(), 1e-3, what="wgrad slab sum vs fp32")


def test_gemm_wgrad_8ph_strided_and_training_dispatch():
    import sdpnet_train as st
    # strided token rows (ld > N), a 40-token partial last K-tile, bit-reproducible
    M, N, K = 4136, 512, 768
    base_dy = rnd(M, N + 64, seed=33, dtype=BF, scale=0.5)
    base_x = rnd(M, K + 8, seed=34, dtype=BF)
    dy, x = base_dy[:, 32:32 + N], base_x[:, :K]
    assert st._wgrad_8ph_ok(dy, x)
    a = st._wgrad(dy, x)
    b = st._wgrad(dy, x)
    assert torch.equal(a, b)
    close(a, dy.float().t() @ x.float(), 1e-5, "wgrad strided + tail")
    old = st._WGRAD_8PH
    try:
        st._WGRAD_8PH = False
        c = st._wgrad(dy.contiguous(), x.contiguous())
    finally:
        st._WGRAD_8PH = old
    close(a, c, 1e-5, "wgrad 8ph vs gemm_flex")


@pytest.mark.parametrize("dtype", [torch.float32, BF])
@pytest.mark.parametrize("eps", [0.0, 0.1])
def test_ce_loss(dtype, eps):
    B, K = 37, 1000
    logits = rnd(B, K, seed=24, dtype=dtype, scale=3)
    labels = torch.randint(0, K, (B,), generator=torch.Generator().manual_seed(0)).to(DEV)
    d = torch.empty_like(logits)
    loss = torch.zeros(1, device=DEV)
    sp.ce_loss(logits, labels, eps, 8.0, d, loss)
    lr = logits.float().clone().requires_grad_(True)
    ref = F.cross_entropy(lr, labels, label_smoothing=eps)
    (g,) = torch.autograd.grad(ref * 8.0, lr)
    close(loss, ref.detach().view(1), 1e-5, "ce loss")
    close(d, g, 1e-5 if dtype == torch.float32 else 2e-2, "ce dlogits")


@pytest.mark.parametrize("dtype", [torch.float32, BF])
@pytest.mark.parametrize("eps", [0.0, 0.1])
def test_ce_loss_soft_targets(dtype, eps):
    # CutMix / MixUp probability targets (dataset_generator.py:105-110) into nn.CrossEntropyLoss
    B, K = 37, 1000
    logits = rnd(B, K, seed=27, dtype=dtype, scale=3)
    g = torch.Generator().manual_seed(1)
    a = torch.randint(0, K, (B,), generator=g)
    b = torch.randint(0, K, (B,), generator=g)
    lam = torch.rand(B, 1, generator=g)
    tgt = (lam * F.one_hot(a, K) + (1 - lam) * F.one_hot(b, K)).float().to(DEV)
    d = torch.empty_like(logits)
    loss = torch.zeros(1, device=DEV)
    sp.ce_loss_soft(logits, tgt, eps, 8.0, d, loss)
    lr = logits.float().clone().requires_grad_(True)
    ref = F.cross_entropy(lr, tgt, label_smoothing=eps)
    (gr,) = torch.autograd.grad(ref * 8.0, lr)
    close(loss, ref.detach().view(1), 1e-5, "soft ce loss")
    close(d, gr, 1e-5 if dtype == torch.float32 else 2e-2, "soft ce dlogits")
    # through the autograd entry point
    import sdpnet_train as st
    lr2 = logits.float().clone().requires_grad_(True)
    l2 = st.cross_entropy(lr2, tgt, label_smoothing=eps)
    l2.backward()
    close(l2.detach().view(1), ref.detach().view(1), 1e-5, "cross_entropy(soft)")
    close(lr2.grad, gr / 8.0, 1e-5, "cross_entropy(soft) grad")


def test_ce_loss_label_out_of_range_is_nan_not_oob():
    B, K = 8, 100
    logits = rnd(B, K, seed=28)
    labels = torch.tensor([0, 5, -7, 99, 100, 3, 7, 1], device=DEV)
    d = torch.empty_like(logits)
    loss = torch.zeros(1, device=DEV)
    sp.ce_loss(logits, labels, 0.0, 1.0, d, loss)
    torch.cuda.synchronize()
    assert torch.isnan(loss).all()
    bad = torch.isnan(d).all(dim=1).cpu()
    assert bad.tolist() == [False, False, True, False, True, False, False, False]


@pytest.mark.parametrize("dtype", [torch.float32, BF])
@pytest.mark.parametrize("eps", [0.0, 0.1])
@pytest.mark.parametrize("ignore", [-100, 3])
def test_ce_loss_ignore_index(dtype, eps, ignore):
    """nn.CrossEntropyLoss's ignore_index (default -100, training_tools.py:72): ignored rows leave
    the loss and the mean's divisor and get zero gradient, against F.cross_entropy; every row
    ignored gives NaN as torch does."""
    import sdpnet_train as st
    B, K = 37, 1000
    logits = rnd(B, K, seed=29, dtype=dtype, scale=3)
    labels = torch.randint(0, K, (B,), generator=torch.Generator().manual_seed(2))
    labels[[0, 5, 6, 20, 36]] = ignore
    labels = labels.to(DEV)
    d = torch.empty_like(logits)
    loss = torch.zeros(1, device=DEV)
    sp.ce_loss(logits, labels, eps, 8.0, d, loss, ignore_index=ignore)
    lr = logits.float().clone().requires_grad_(True)
    ref = F.cross_entropy(lr, labels, label_smoothing=eps, ignore_index=ignore)
    (g,) = torch.autograd.grad(ref * 8.0, lr)
    close(loss, ref.detach().view(1), 1e-5, "ce loss (ignore_index)")
    close(d, g, 1e-5 if dtype == torch.float32 else 2e-2, "ce dlogits (ignore_index)")
    assert (d[[0, 5, 6, 20, 36]] == 0).all()
    lr2 = logits.float().clone().requires_grad_(True)
    l2 = st.cross_entropy(lr2, labels, label_smoothing=eps, ignore_index=ignore)
    l2.backward()
    close(l2.detach().view(1), ref.detach().view(1), 1e-5, "cross_entropy(ignore_index)")
    close(lr2.grad, g / 8.0, 1e-5, "cross_entropy(ignore_index) grad")
    # every row ignored: torch's mean is 0 / 0
    loss.zero_()
    sp.ce_loss(logits, torch.full((B,), ignore, device=DEV), eps, 1.0, d, loss, ignore_index=ignore)
    torch.cuda.synchronize()
    assert torch.isnan(loss).all() and (d == 0).all()


@pytest.mark.parametrize("xdt,ydt", [(BF, torch.float32), (BF, BF), (torch.float32, BF)])
@pytest.mark.parametrize("with_scale", [False, True])
def test_rowscale_dropout_fused_is_bit_identical(xdt, ydt, with_scale):
    # EncoderLayer's x + drop_path(dropout(proj)) (mode 1) and its gradient cast into the branch
    # (mode 2) in one pass == act_fwd / act_bwd (dropout only) + rowscale_add, bit for bit
    M, N, grp, p, seed = 780, 768, 260, 0.2, 12345
    x = rnd(M, N, seed=60, dtype=xdt)
    r = rnd(M, N, seed=61, dtype=ydt)
    sc = (torch.rand(M // grp, generator=torch.Generator().manual_seed(2)) + 0.5).to(DEV) if with_scale else None
    if xdt == BF:  # mode 1: branch x (bf16) into the stream (ydt) with the residual
        got = torch.empty(M, N, dtype=ydt, device=DEV)
        sp.rowscale_add(sp.dense(x), sp.dense(got), M, N, scale=sc, sgrp=grp, resid=sp.dense(r), p=p, seed=seed,
                        dmode=1)
        tmp = torch.empty_like(x)
        sp.act_fwd(x, tmp, M, N, 0, p, seed)
        ref = torch.empty(M, N, dtype=ydt, device=DEV)
        sp.rowscale_add(sp.dense(tmp), sp.dense(ref), M, N, scale=sc, sgrp=grp, resid=sp.dense(r))
        assert torch.equal(got, ref)
        assert 0.15 < float((tmp == 0).float().mean()) < 0.25
    # mode 2: x cast into a bf16 branch, then the dropout mask on the rounded value
    got = torch.empty(M, N, dtype=ydt, device=DEV)
    sp.rowscale_add(sp.dense(x), sp.dense(got), M, N, scale=sc, sgrp=grp, p=p, seed=seed, dmode=2)
    ref = torch.empty(M, N, dtype=ydt, device=DEV)
    sp.rowscale_add(sp.dense(x), sp.dense(ref), M, N, scale=sc, sgrp=grp)
    sp.act_bwd(ref, ref, ref, M, N, 0, p, seed)
    assert torch.equal(got, ref)


def test_mt_cast_transpose():
    # one launch, ragged shapes, a stacked destination (the fused q/k/v weight) and NULL outputs
    shapes = [(768, 768), (100, 70), (768, 588), (3, 130), (64, 64)]
    srcs = [rnd(r, c, seed=40 + i) for i, (r, c) in enumerate(shapes)]
    jobs, outs = [], []
    for i, x in enumerate(srcs):
        d = torch.zeros(x.shape, dtype=BF, device=DEV) if i != 3 else None
        t = torch.zeros(x.shape[::-1], dtype=BF, device=DEV) if i != 4 else None
        jobs.append((x, d, t))
        outs.append((d, t))
    stacked = torch.zeros(3 * 256, 256, dtype=BF, device=DEV)
    stacked_t = torch.zeros(256, 3 * 256, dtype=BF, device=DEV)
    parts = [rnd(256, 256, seed=50 + j) for j in range(3)]
    for j, x in enumerate(parts):
        jobs.append((x, stacked[j * 256:(j + 1) * 256], stacked_t[:, j * 256:(j + 1) * 256]))
    sp.mt_cast_transpose(jobs)
    for x, (d, t) in zip(srcs, outs):
        if d is not None:
            assert torch.equal(d, x.to(BF))
        if t is not None:
            assert torch.equal(t, x.to(BF).t())
    ref = torch.cat(parts, 0).to(BF)
    assert torch.equal(stacked, ref) and torch.equal(stacked_t, ref.t())


@pytest.mark.parametrize("dtype", [torch.float32, BF])
@pytest.mark.parametrize("R,C", [(768, 3072), (100, 37), (1, 64)])
def test_transpose(dtype, R, C):
    x = rnd(R, C, seed=25, dtype=dtype)
    assert torch.equal(sp.transpose(x), x.t().contiguous())
    y = rnd(R, C + 6, seed=26, dtype=dtype)[:, 3:3 + C]  # strided rows
    assert torch.equal(sp.transpose(y), y.t().contiguous())


@pytest.mark.parametrize("dtype", [torch.float32, BF])
@pytest.mark.parametrize("M,C", [(300, 768), (77, 96), (5, 1024), (9, 2048), (61, 64), (1, 128), (130, 16)])
def test_ln_fwd_one_pass(dtype, M, C):
    x = (rnd(M, C, seed=27, scale=1.5) + rnd(M, 1, seed=28, scale=2)).to(dtype)
    g, b = rnd(C, seed=29) * 0.2 + 1, rnd(C, seed=30) * 0.2
    st = torch.empty(M, 2, device=DEV)
    y = torch.empty_like(x)
    sp.ln_fwd(sp.dense(x), 1e-5, g, b, st, sp.dense(y), M, C)
    xf = x.float()
    close(st[:, 0], xf.mean(1), 1e-5, "mean")
    close(st[:, 1], 1 / torch.sqrt(xf.var(1, unbiased=False) + 1e-5), 1e-4, "rstd")
    close(y, F.layer_norm(xf, (C,), g, b, 1e-5), 2e-5 if dtype == torch.float32 else 2e-2, "ln_fwd")


@pytest.mark.parametrize("dtype", [torch.float32, BF])
def test_head_layernorm_on_qkv_rows(dtype):
    """The training q/k LayerNorm: per-head rows of hd = 96 inside a [T, 3C] QKV buffer
    (Rows(qkv, hd, H, 3H, off)), several heads per wave (ln_fwd_sm / ln_bwd_sm)."""
    T, H, hd, eps = 1001, 8, 96, 1e-5
    C = H * hd
    qkv = rnd(T, 3 * C, seed=31, dtype=dtype, scale=1.5)
    g, b = rnd(hd, seed=32) * 0.2 + 1, rnd(hd, seed=33) * 0.2
    out = torch.zeros_like(qkv)
    st = torch.empty(T * H, 2, device=DEV)
    sp.ln_fwd(sp.Rows(qkv, hd, H, 3 * H, H), eps, g, b, st, sp.Rows(out, hd, H, 3 * H, H), T * H, hd)
    k = qkv[:, C:2 * C].float().reshape(T, H, hd)
    kr = k.clone().requires_grad_(True)
    ref = F.layer_norm(kr, (hd,), g, b, eps)
    close(out[:, C:2 * C].reshape(T, H, hd), ref.detach(), 2e-5 if dtype == torch.float32 else 2e-2, "head ln fwd")
    assert (out[:, :C] == 0).all() and (out[:, 2 * C:] == 0).all()
    dy = torch.zeros_like(qkv)
    dy[:, C:2 * C] = rnd(T, C, seed=34, dtype=dtype)
    dx = torch.zeros_like(qkv)
    dg, db = sp.ln_bwd(sp.Rows(qkv, hd, H, 3 * H, H), st, g, sp.Rows(dy, hd, H, 3 * H, H),
                       sp.Rows(dx, hd, H, 3 * H, H), T * H, hd)
    gx, = torch.autograd.grad(ref, kr, dy[:, C:2 * C].float().reshape(T, H, hd))
    tol = 8e-5 if dtype == torch.float32 else 8e-2
    close(dx[:, C:2 * C].reshape(T, H, hd), gx, tol, "head ln dx")
    xh = (k - k.mean(-1, keepdim=True)) / torch.sqrt(k.var(-1, unbiased=False, keepdim=True) + eps)
    close(dg, (dy[:, C:2 * C].float().reshape(T, H, hd) * xh).sum((0, 1)), tol * 10, "head ln dgamma")
    close(db, dy[:, C:2 * C].float().reshape(T, H, hd).sum((0, 1)), tol * 10, "head ln dbeta")


@pytest.mark.parametrize("dtype", [torch.float32, BF])
@pytest.mark.parametrize("act", [1, 2, 7])
@pytest.mark.parametrize("C", [64, 36])   # 8-wide kernel / scalar kernel
def test_act_rowscale_add_matches_two_passes(dtype, act, C):
    """sdp_act_rowscale_add == sdp_act_fwd then sdp_rowscale_add, bit for bit (token row maps)."""
    B, R, P = 3, 2, 49
    N = R + P
    z = rnd(B * P, C, seed=50, dtype=dtype)
    tok = rnd(B * N, C, seed=51, dtype=dtype)
    scale = torch.rand(B, generator=torch.Generator().manual_seed(52)).to(DEV) + 0.5
    h = torch.empty_like(z)
    sp.act_fwd(z, h, B * P, C, act)
    ref = torch.zeros(B * N, C, dtype=dtype, device=DEV)
    sp.rowscale_add(sp.dense(h), sp.Rows(ref, C, P, N, R), B * P, C, scale=scale, sgrp=P, resid=sp.Rows(tok, C, P, N, R))
    got = torch.zeros_like(ref)
    sp.rowscale_add(sp.dense(z), sp.Rows(got, C, P, N, R), B * P, C, scale=scale, sgrp=P,
                    resid=sp.Rows(tok, C, P, N, R), act=act)
    assert torch.equal(got, ref)


# ------------------------------------------------- flash training attention (attn_train.hip)
@pytest.mark.parametrize("B,N,H,hd", [(2, 260, 8, 96), (3, 200, 8, 96), (2, 53, 4, 16), (1, 77, 2, 64),
                                      (1, 33, 2, 128), (2, 100, 4, 48), (1, 1, 2, 32), (2, 300, 2, 80),
                                      (1, 700, 2, 96), (1, 64, 2, 96), (1, 96, 1, 128)])
@pytest.mark.parametrize("p", [0.0, 0.2])
def test_flash_train_attention_vs_torch(B, N, H, hd, p):
    """O, the row LSE and dQ / dK / dV of the flash training kernels against torch fp32 autograd of
    dropout(softmax(QK^T / sqrt(hd))) V on the same bf16 inputs, with the kernels' own dropout mask
    (sdp_attn_dropout_mask) -- layers.py:289-291.  Tolerance: bf16 operand / P rounding, 2e-2 of the
    tensor's max |.| (O 1e-2); LSE 1e-4 relative."""
    assert sp.attn_train_applies(BF, N, hd)
    C = H * hd
    T = B * N
    qkv = rnd(T, 3 * C, seed=1, scale=1.5).to(BF)
    do = rnd(T, C, seed=2).to(BF)
    seed = 1234567 + N
    o = torch.empty(T, C, dtype=BF, device=DEV)
    lse = torch.empty(B * H * N, dtype=torch.float32, device=DEV)
    scale = 1.0 / math.sqrt(hd)
    sp.attn_train_fwd(qkv, o, lse, B, N, H, hd, scale, p, seed)
    dqkv = torch.full((T, 3 * C), float("nan"), dtype=BF, device=DEV)
    delta = torch.empty(B * H * N, dtype=torch.float32, device=DEV)
    sp.attn_train_bwd(qkv, o, do, lse, delta, (dqkv, 0), (dqkv, C), (dqkv, 2 * C), B, N, H, hd, scale, p, seed)
    # reference
    x = qkv.float().view(B, N, 3, H, hd).permute(2, 0, 3, 1, 4)  # [3, B, H, N, hd]
    q, k, v = (t.clone().requires_grad_(True) for t in x)
    s = q @ k.transpose(-1, -2) * scale
    P = torch.softmax(s, -1)
    mask = sp.attn_dropout_mask(B * H, N, p, seed, DEV).view(B, H, N, N).float()
    if p > 0:
        assert abs(float(mask.mean()) - (1 - p)) < 0.05 + 3.0 / math.sqrt(mask.numel())
    Pd = P * mask / (1 - p)
    ref_o = Pd @ v
    ref_o.backward(do.float().view(B, N, H, hd).permute(0, 2, 1, 3))
    close(o.float().view(B, N, H, hd).permute(0, 2, 1, 3), ref_o.detach(), 1e-2, "O")
    ref_lse2 = torch.logsumexp(s.detach(), -1) / math.log(2.0)
    close(lse.view(B, H, N), ref_lse2, 1e-4, "lse")
    g = dqkv.float().view(B, N, 3, H, hd).permute(2, 0, 3, 1, 4)
    close(g[2], v.grad, 2e-2, "dV")
    # dQ / dK are judged on the gradient scale of the layer (dV's): D = rowsum(dO o O) uses the
    # bf16-rounded O, so where the exact dS is 0 (N = 1: softmax of one key) ours is rounding noise
    gs = max(1.0, float(v.grad.abs().max()))
    for got, ref, what in ((g[0], q.grad, "dQ"), (g[1], k.grad, "dK")):
        err = float((got - ref).abs().max())
        assert err <= 2e-2 * max(gs, float(ref.abs().max())), f"{what}: {err:.3e} (scale {gs:.3e})"


@pytest.mark.parametrize("act", ["gelu", "relu", "kelu"])
@pytest.mark.parametrize("p", [0.0, 0.2])
@pytest.mark.parametrize("M,N,K", [(512, 3072, 768), (300, 256, 128), (1000, 1024, 256)])
def test_gemm_train_epilogues_bit_identical_to_separate_kernels(act, p, M, N, K):
    """sdp_gemm_train_epi: mode 1 (z and dropout(act(z)) from one launch) and mode 2
    (dropout(dy . w^T) * act'(z)) equal the fast GEMM followed by sdp_act_fwd / sdp_act_bwd bit
    for bit (same masks), ragged M included."""
    code = sp.ACT_CODES[act]
    x, w = rnd(M, K, seed=1, dtype=BF), rnd(N, K, seed=2, dtype=BF, scale=0.05)
    b = rnd(N, seed=3, scale=0.1)
    z, h = torch.empty(M, N, dtype=BF, device=DEV), torch.empty(M, N, dtype=BF, device=DEV)
    assert sp.gemm_train_epi(1, x, w, z, M, N, K, bias=b, y2=h, act=code, p=p, seed=77)
    z_ref, h_ref = torch.empty_like(z), torch.empty_like(h)
    sp.gemm(sp.dense(x), w, sp.dense(z_ref), M, N, K, bias=b)
    sp.act_fwd(z_ref, h_ref, M, N, code, p, 77)
    assert torch.equal(z, z_ref) and torch.equal(h, h_ref)
    # mode 2: dy [M, K2] . wt^T with wt [N, K2] -> [M, N], times act'(z)
    K2 = 256
    dy, wt = rnd(M, K2, seed=4, dtype=BF), rnd(N, K2, seed=5, dtype=BF, scale=0.05)
    dz = torch.empty(M, N, dtype=BF, device=DEV)
    assert sp.gemm_train_epi(2, dy, wt, dz, M, N, K2, z=z, act=code, p=p, seed=78)
    dh = torch.empty(M, N, dtype=BF, device=DEV)
    sp.gemm(sp.dense(dy), wt, sp.dense(dh), M, N, K2)
    dz_ref = torch.empty_like(dz)
    sp.act_bwd(z, dh, dz_ref, M, N, code, p, 78)
    assert torch.equal(dz, dz_ref)
    # shapes the fast kernel does not take are refused without a launch
    assert not sp.gemm_train_epi(1, x[:100].contiguous(), w, z[:100].contiguous(), 100, N, K, bias=b,
                                 y2=h[:100].contiguous(), act=code)


@pytest.mark.parametrize("xdt,ydt,adt", [(BF, torch.float32, BF), (BF, BF, BF), (torch.float32, torch.float32,
                                                                            torch.float32)])
@pytest.mark.parametrize("act,p", [(0, 0.0), (1, 0.0), (0, 0.2)])
@pytest.mark.parametrize("C", [768, 96, 1032])
def test_add_ln_fwd_one_pass_is_bit_identical(xdt, ydt, adt, act, p, C):
    """sdp_add_ln_fwd (the branch add x + drop_path(act / dropout(z)) and the next LayerNorm in one
    pass) stores the same sum, the same statistics and the same normalised rows as
    sdp_rowscale_add[_mixed / _dropout] followed by sdp_ln_fwd[_mixed] -- on the token buffer's image
    rows (row maps), with a drop-path scale per image, every dtype mix the training step uses."""
    if p > 0 and act:
        pytest.skip("the dropout branch carries no activation (EncoderLayer o_proj)")
    B, R, P = 3, 4, 49
    N = R + P
    M = B * P
    z = rnd(M, C, seed=71, dtype=xdt)
    tok = rnd(B * N, C, seed=72, dtype=ydt, scale=2.0) + 0.5
    g, b = rnd(C, seed=73) * 0.2 + 1, rnd(C, seed=74) * 0.2
    scale = torch.tensor([1.25, 0.0, 1.25], device=DEV)
    outs = []
    for fused in (False, True):
        y = torch.full((B * N, C), float("nan"), dtype=ydt, device=DEV)
        a = torch.full((M, C), float("nan"), dtype=adt, device=DEV)
        st = torch.full((M, 2), float("nan"), device=DEV)
        img, res = sp.Rows(y, C, P, N, R), sp.Rows(tok, C, P, N, R)
        kw = dict(scale=scale, sgrp=P, act=act, p=p, seed=1234, dmode=1 if p > 0 else 0)
        if fused and sp.add_ln_fwd(sp.dense(z), img, sp.dense(a), M, C, res, 1e-5, g, b, st, **kw):
            assert C > 128
        else:
            assert not fused or C <= 128  # short rows: the two passes (ln_fwd's several-rows-per-wave kernel)
            sp.rowscale_add(sp.dense(z), img, M, C, resid=res, **kw)
            sp.ln_fwd(img, 1e-5, g, b, st, sp.dense(a), M, C)
        torch.cuda.synchronize()
        outs.append((y.view(B, N, C)[:, R:], a, st))
    for u, v in zip(outs[0], outs[1]):
        assert torch.equal(u, v)
    # against plain torch: LN of the stored sum
    ys = outs[1][0].reshape(M, C).float()
    close(outs[1][1], F.layer_norm(ys, (C,), g, b, 1e-5), 1e-2 if adt == BF else 1e-5, what="add_ln_fwd LN")


def _ln_bwd_case(B, R, P, C, seed, dense_rows):
    N = R + P
    M = B * P
    x = rnd(B, N, C, seed=seed, scale=1.5) + rnd(B, N, 1, seed=seed + 1, scale=2)
    add = rnd(B, N, C, seed=seed + 2)
    da = rnd(M, C, seed=seed + 3, dtype=BF)
    g = rnd(C, seed=seed + 4) * 0.2 + 1
    st = torch.empty(M, 2, device=DEV)
    rows = (lambda t: sp.dense(t.view(-1, C))) if dense_rows else (lambda t: sp.Rows(t, C, P, N, R))
    if dense_rows:
        M = B * N
        da = rnd(M, C, seed=seed + 3, dtype=BF)
        st = torch.empty(M, 2, device=DEV)
    sp.rowstats(rows(x), 1e-6, st, M, C)
    return x, add, da, g, st, rows, M


@pytest.mark.parametrize("ticket", [False, True])
@pytest.mark.parametrize("C", [768, 1032])
@pytest.mark.parametrize("style", ["mixer", "encoder"])
def test_ln_bwd_fused_matches_separate_passes(style, C, ticket, monkeypatch):
    """sdp_ln_bwd_fused: DX and the emitted branch gradient bit-identical to sdp_ln_bwd_mixed followed by
    the rowscale (drop path / dropout mode 2) and act_bwd passes; the in-kernel affine sums (ticketed,
    fixed order) agree with the two-level seg_colsum sums to fp32 rounding and repeat bit for bit
    (the tickets reset themselves between launches)."""
    B, R, P = (3, 4, 49) if style == "mixer" else (5, 1, 63)
    x, add, da, g, st, rows, M = _ln_bwd_case(B, R, P, C, 50, style == "encoder")
    N = R + P
    if style == "mixer":
        scale, sgrp = torch.tensor([1.25, 0.0, 1.25], device=DEV), P
        z = rnd(M, C, seed=57, dtype=BF)
        emit = dict(scale=scale, sgrp=sgrp, z=z, act=1)
    else:
        scale, sgrp = torch.tensor([1.25, 0.0, 1.25, 1.25, 1.25], device=DEV), N
        emit = dict(scale=scale, sgrp=sgrp, p=0.2, seed=321, dmode=2)
    outs = []
    monkeypatch.setattr(sp, "_LN_TICKET", ticket)
    for fused in (False, True, True):
        monkeypatch.setattr(sp, "_LN_BWD_FUSED", fused)
        dx = torch.zeros_like(x)
        o2 = torch.empty(M, C, device=DEV, dtype=BF)
        aff = sp.ln_bwd(rows(x), st, g, sp.dense(da), rows(dx), M, C, add=rows(add), emit=dict(emit, out=o2))
        outs.append((dx, o2, aff))
    (dx0, o0, (g0, b0)), (dx1, o1, (g1, b1)), (dx2, o2_, (g2, b2)) = outs
    assert torch.equal(dx0, dx1) and torch.equal(o0, o1)
    assert torch.equal(g1, g2) and torch.equal(b1, b2)
    close(g1, g0, 1e-5, "dgamma")
    close(b1, b0, 1e-5, "dbeta")
    ref_b = da.float().sum(0)
    close(b1, ref_b, 1e-4, "dbeta vs torch")


def test_ln_bwd_fused_affine_full_grid_deterministic(monkeypatch):
    """1024 blocks (32 ticket groups) at the XL training shape: the affine sums equal the two-level
    path to fp32 rounding, repeat bit for bit, and the branch-free call (no emit) leaves dx as before."""
    B, R, P, C = 120, 4, 256, 768
    x, add, da, g, st, rows, M = _ln_bwd_case(B, R, P, C, 60, False)
    monkeypatch.setattr(sp, "_LN_TICKET", True)
    res = []
    for fused in (False, True, True):
        monkeypatch.setattr(sp, "_LN_BWD_FUSED", fused)
        dx = torch.zeros_like(x)
        res.append((dx, sp.ln_bwd(rows(x), st, g, sp.dense(da), rows(dx), M, C, add=rows(add))))
    (d0, (g0, b0)), (d1, (g1, b1)), (d2, (g2, b2)) = res
    assert torch.equal(d0, d1)
    assert torch.equal(g1, g2) and torch.equal(b1, b2)
    close(g1, g0, 1e-5, "dgamma")
    close(b1, b0, 1e-5, "dbeta")


@pytest.mark.parametrize("C", [768, 96])
@pytest.mark.parametrize("R", [0, 4])
def test_register_rows_copied_in_the_row_kernels(R, C):
    """The register-row copy jobs folded into sdp_add_ln_fwd (two destinations) and sdp_ln_bwd_fused
    (one): register rows equal the source's, image rows are the kernels' own results.  C = 96: the
    one-launch forms do not apply and the wrappers' separate copies run instead."""
    import sdpnet_train as st_
    B, P = 3, 49
    N, M = R + P, B * P
    tok = rnd(B, N, C, seed=70)
    z = rnd(M, C, seed=71, dtype=BF)
    g, b = rnd(C, seed=72) * 0.2 + 1, rnd(C, seed=73) * 0.2
    mid, out = torch.full_like(tok, float("nan")), torch.full_like(tok, float("nan"))
    img = lambda t: sp.Rows(t, C, P, N, R)  # noqa: E731
    a, st = st_._add_ln_fwd(sp.dense(z), img(mid), M, C, img(tok), g, b, 1e-6, BF, act=1,
                            regs=(tok, [mid, out], B, R, N) if R else None)
    assert torch.equal(mid[:, :R], tok[:, :R]) and torch.equal(out[:, :R], tok[:, :R])
    assert not torch.isnan(mid[:, R:]).any() and torch.isnan(out[:, R:]).all()
    da = rnd(M, C, seed=74, dtype=BF)
    dmid = torch.full_like(tok, float("nan"))
    dz = torch.empty(M, C, device=DEV, dtype=BF)
    sp.ln_bwd(img(mid), st, g, sp.dense(da), img(dmid), M, C, add=img(tok), emit=dict(out=dz, z=z, act=1),
              regs=(tok, [dmid], B, R, N) if R else None)
    assert torch.equal(dmid[:, :R], tok[:, :R]) and not torch.isnan(dmid).any()
