"""bf16 training-gradient error budget for the train fixtures (diagnostic, GPU box).

For each case: our bf16 path (fp32 stream and bf16 stream) against the reference's fp32
gradient, next to the reference's own CPU-autocast error (fixture grad_ac/*) and the same
restated reference (oracle) run under CUDA autocast on the GPU.  Prints the worst tensors.
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "sdp-net_amd")]
import golden_util as gu  # noqa: E402
import sdpnet_oracle as orc  # noqa: E402
import synth  # noqa: E402
import test_train as tt  # noqa: E402


def main():
    import sdpnet_train
    for name in tt.CASES:
        meta, arr, m, sd, x, y = tt._case(name)
        fl = tt._floor(arr)
        keys = [k for k, _ in m.named_parameters()]
        osd = {k: v.cuda().clone().requires_grad_(v.is_floating_point()) for k, v in sd.items()}
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lo = F.cross_entropy(orc.forward.__wrapped__(x.cuda(), osd, meta["config"],
                                                         num_registers=meta["num_registers"]).float(),
                                 y.cuda(), label_smoothing=meta["label_smoothing"])
        lo.backward()
        rows = {}
        for k in keys:
            ref = arr["grad/" + k]
            rows[k] = [tt._rel(arr["grad_ac/" + k], ref, fl), tt._rel(osd[k].grad.float().cpu().numpy(), ref, fl)]
        for fs in (True, False):
            _, _, mm, _, _ = tt._train_step(name, True, fp32_stream=fs)
            for k, p in mm.named_parameters():
                rows[k].append(tt._rel(p.grad.cpu().numpy(), arr["grad/" + k], fl))
        order = sorted(keys, key=lambda k: -rows[k][2] / max(rows[k][0], 1e-9))
        print(f"== {name}: rel error vs reference fp32 grads  [ref CPU autocast | ref CUDA autocast | ours fp32-stream"
              f" | ours bf16-stream]")
        for k in order[:10]:
            a, b, c, d = rows[k]
            print(f"  {k:55s} {a:.2e} {b:.2e} {c:.2e} {d:.2e}   ours/cpu {c / max(a, 1e-12):5.2f}"
                  f"  ours/max {c / max(a, b, 1e-12):5.2f}")


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def seeds_sweep(name="train_tf_bias_pool", n=12):
    """Same weights, n random input batches: distribution of the per-tensor error of ours
    (fp32 stream) and of the reference restatement under CUDA autocast, both against fp32
    autograd of the reference restatement on the GPU."""
    import model as ours
    meta, arr, m0, sd, x0, y0 = tt._case(name)
    cfg = meta["config"]
    keys = [k for k, _ in m0.named_parameters()]
    m = m0.cuda().train()
    ratios = {k: [] for k in keys}
    errs = {k: [] for k in keys}
    for s in range(n):
        x = synth.synth_images(100 + s, meta["batch"], meta["image"]).cuda()
        y = torch.randint(0, cfg["output_classes"], (meta["batch"],), generator=torch.Generator().manual_seed(s)).cuda()
        g = {}
        for ac in (False, True):
            osd = {k: v.cuda().clone().requires_grad_(v.is_floating_point()) for k, v in sd.items()}
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=ac):
                lo = F.cross_entropy(orc.forward.__wrapped__(x, osd, cfg, num_registers=meta["num_registers"]).float(),
                                     y, label_smoothing=meta["label_smoothing"])
            lo.backward()
            g[ac] = {k: osd[k].grad.float().cpu().numpy() for k in keys}
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            import sdpnet_train
            loss = sdpnet_train.cross_entropy(m(x, num_registers=meta["num_registers"]), y, meta["label_smoothing"])
        loss.backward()
        fl = 1e-3 * max(float(np.abs(v).max()) for v in g[False].values())
        for k, p in m.named_parameters():
            a = tt._rel(g[True][k], g[False][k], fl)
            c = tt._rel(p.grad.cpu().numpy(), g[False][k], fl)
            errs[k].append((a, c))
            ratios[k].append(c / max(a, 1e-12))
    order = sorted(keys, key=lambda k: -np.median(ratios[k]))
    print(f"== {name}: {n} input batches; median rel error [ref CUDA autocast | ours], median / max of ours/ref")
    for k in order[:8]:
        e = np.array(errs[k])
        print(f"  {k:55s} {np.median(e[:, 0]):.2e} {np.median(e[:, 1]):.2e}   median ratio "
              f"{np.median(ratios[k]):.2f}  max ratio {np.max(ratios[k]):.2f}")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "sweep":
    seeds_sweep()
