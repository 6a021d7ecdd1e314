"""Generate the TRAINING-step golden fixtures under tests/golden/ — CONTAINER-ONLY tool.

Imports the reference (/root/reference, read-only) the same way gen_golden.py does (empty
``wandb`` stub) and records, for small configurations with dropout and stochastic depth
off (their RNG streams cannot be reproduced), the reference's own:

  * training-mode loss: nn.CrossEntropyLoss(label_smoothing=0.1) (training_tools.py:76, :88)
    of ``model.train()`` logits on synthetic images and labels;
  * the fp32 gradient of every parameter after ``loss.backward()`` (training_tools.py:91),
    and the same under CPU bf16 autocast (the reference's training dtype) as the error yardstick
    of the bf16 path;
  * the clip_grad_norm_(5) total norm (training_tools.py:97) and one
    torch.optim.AdamW(lr, weight_decay) step (training_tools.py:235, :98) -> parameters.

It first checks the build's CPU oracle (autograd through oracle/sdpnet_oracle.py's
forward) against the reference's gradients (<= 1e-5 relative), then writes the fixtures.
Nothing from /root/reference is copied: fixtures are data (inputs are regenerated from
seeds on the GPU box, outputs are stored).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_train_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import synth  # noqa: E402
import sdpnet_oracle as orc  # noqa: E402
from gen_golden import import_reference, weights_digest, WSEED, XSEED  # noqa: E402

BASE = dict(embedding_dim=32, num_blocks=2, n_head=4, conv_kernel_size=7, patch_size=16, max_image_size=[16, 16],
            output_classes=10, head_output_from_register=True, conv_first=True, ffn_dropout=0.0, attn_dropout=0.0)
# name -> (config, batch, image size, num_registers)
CASES = {
    "train_cf": (dict(BASE), 3, 64, 3),
    "train_tf_bias_pool": (dict(BASE, conv_first=False, mixer_ffn_bias=True, mixer_deptwise_bias=True,
                                output_head_bias=True, head_output_from_register=False, conv_kernel_size=5,
                                activation="relu"), 2, 64, 3),
}
LABEL_SMOOTHING, LR, WD, MAX_NORM = 0.1, 1e-3, 0.05, 5.0


def labels_for(name: str, B: int, K: int) -> torch.Tensor:
    return torch.from_numpy((synth.uniform(synth.key_seed(7, name), B) * K).astype(np.int64))


def main():
    ref_model, _, _ = import_reference()
    torch.set_num_threads(8)
    man = {}
    for name, (cfg, B, img, nreg) in CASES.items():
        torch.manual_seed(0)
        m = ref_model.MainModel.from_dict(**cfg)
        sd = synth.synth_state_dict(m, WSEED)
        m.load_state_dict(sd)
        m.train()
        x = synth.synth_images(XSEED, B, img)
        y = labels_for(name, B, cfg["output_classes"])
        logits = m(x.clone(), num_registers=nreg)
        loss = F.cross_entropy(logits, y, label_smoothing=LABEL_SMOOTHING)
        loss.backward()
        grads = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
        # oracle: autograd through the CPU restatement's forward (no grad-disabling decorator)
        osd = {k: v.clone().requires_grad_(v.is_floating_point()) for k, v in sd.items()}
        olog = orc.forward.__wrapped__(x.clone(), osd, cfg, num_registers=nreg)
        oloss = F.cross_entropy(olog, y, label_smoothing=LABEL_SMOOTHING)
        oloss.backward()
        worst = 0.0
        for k, g in grads.items():
            og = osd[k].grad
            og = torch.zeros_like(g) if og is None else og
            worst = max(worst, float((og - g).abs().max()) / max(1e-12, float(g.abs().max())))
        assert worst <= 1e-4 and abs(float(oloss) - float(loss)) <= 1e-6, (name, worst)
        # the reference's own bf16 training forward (CPU autocast, training_tools.py:85): its
        # gradient error is the yardstick for our bf16 path
        m.zero_grad(set_to_none=True)
        with torch.autocast("cpu", dtype=torch.bfloat16):
            lac = F.cross_entropy(m(x.clone(), num_registers=nreg), y, label_smoothing=LABEL_SMOOTHING)
        lac.backward()
        grads_ac = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
        for k, p in m.named_parameters():
            p.grad = grads[k].clone()
        total_norm = float(torch.nn.utils.clip_grad_norm_(m.parameters(), MAX_NORM))
        opt = torch.optim.AdamW(m.parameters(), lr=LR, weight_decay=WD)
        opt.step()
        rec = dict(loss=np.float32(loss.item()), logits=logits.detach().numpy(), labels=y.numpy(),
                   total_norm=np.float32(total_norm))
        for k, g in grads.items():
            rec["grad/" + k] = g.numpy()
            rec["grad_ac/" + k] = grads_ac[k].float().numpy()
        rec["loss_ac"] = np.float32(lac.item())
        for k, p in m.named_parameters():
            rec["step/" + k] = p.detach().numpy()
        meta = dict(config=cfg, batch=B, image=img, num_registers=nreg, wseed=WSEED, xseed=XSEED,
                    weights_sha256=weights_digest(sd), label_smoothing=LABEL_SMOOTHING, lr=LR, weight_decay=WD,
                    max_norm=MAX_NORM, oracle_vs_reference_grad_rel=worst)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), meta=json.dumps(meta), **rec)
        man[name] = meta
        print(f"{name}: loss {loss.item():.5f} grad norm {total_norm:.4f} oracle grad rel err {worst:.1e}", flush=True)
    with open(os.path.join(HERE, "TRAIN_MANIFEST.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
