import sys, os, torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "sdp-net_amd"))
import sdpnet_hip as sp
torch.manual_seed(0)
dev = "cuda"
BF = torch.bfloat16
for (M, N, K, dense) in [(600, 768, 768, True), (600, 768, 768, False), (256, 256, 64, True)]:
    x = torch.randn(M, K, device=dev).to(BF)
    w = (torch.randn(N, K, device=dev) * 0.05).to(BF)
    r0 = torch.randn(M, N, device=dev).to(BF)
    res = []
    for spec in (0, 1):
        sp.lib().sdp_gemm_set_epi_spec(spec)
        y = r0.clone()
        part = torch.full((M, N // 64, 2), float("nan"), device=dev)
        if dense:
            sp.gemm(sp.dense(x), w, sp.dense(y), M, N, K, resid=sp.dense(y), act=1, part=part)
        else:
            sp.gemm(sp.dense(x), w, sp.dense(y), M, N, K, resid=None, act=1, part=part)
        torch.cuda.synchronize()
        res.append((y.float(), part))
    (y0, p0), (y1, p1) = res
    d = (y0 - y1).abs()
    print(M, N, K, "dense-resid" if dense else "no-resid", "out maxdiff", d.max().item(), "rows differing", int((d.amax(1) > 0).sum()))
    if (d > 0).any():
        idx = (d > 0).nonzero()[:5]
        print("  first diffs", idx.tolist())
    pd = (p0 - p1).abs()
    print("  part mean maxdiff", pd[..., 0].max().item(), "M2 maxdiff", pd[..., 1].max().item(), "nan in p1", int(torch.isnan(p1).sum()))
    bad = (pd[..., 0] > 1e-4).nonzero()[:8]
    print("  first bad partial (row, chunk)", bad.tolist())
    if len(bad):
        rr, cc = bad[0].tolist()
        print("  p0", p0[rr, cc].tolist(), "p1", p1[rr, cc].tolist(), "true", y1[rr, 64*cc:64*cc+64].mean().item())
