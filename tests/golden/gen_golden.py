"""Generate the golden fixtures under tests/golden/ — CONTAINER-ONLY tool.

Imports the reference (/root/reference, read-only) with an empty ``wandb`` stub
(model.py:11 -> training_utilities.py:7 import it; nothing on the forward path
uses it), loads synthetic weights from ``synth.py`` through ``load_state_dict``
and records the reference's own eval-mode outputs:

  * fp32 logits (the 1e-3 parity target) and CPU-autocast-bf16 logits (what the
    reference calls its bf16 forward, training_tools.py:85) for informational
    error budgets;
  * ``return_raw_outputs`` tensors (x NCHW, registers) for small configs;
  * module-level fixtures (KeLu grid, channel LayerNorm, ConvMixer,
    EncoderLayer incl. mask / manual-softmax path).

It also asserts that the build's CPU oracle (oracle/sdpnet_oracle.py) matches
the reference to <= 1e-5 on every case before writing anything.

Nothing from /root/reference is copied: the fixtures are data (inputs are
regenerated from seeds, outputs are stored).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import synth  # noqa: E402
import sdpnet_oracle as orc  # noqa: E402

REF = "/root/reference"


def import_reference():
    sys.dont_write_bytecode = True
    sys.modules.setdefault("wandb", types.ModuleType("wandb"))
    sys.path.insert(0, REF)
    import model as ref_model  # noqa
    import layers as ref_layers  # noqa
    import training_utilities as ref_tu  # noqa
    sys.path.remove(REF)
    return ref_model, ref_layers, ref_tu


def weights_digest(sd) -> str:
    h = hashlib.sha256()
    for k, v in sd.items():
        h.update(k.encode())
        h.update(v.detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


SMALL = dict(embedding_dim=64, num_blocks=2, n_head=4, conv_kernel_size=7, patch_size=16,
             max_image_size=[16, 16], head_output_from_register=True, conv_first=True,
             ffn_dropout=0.2, attn_dropout=0.2)

# name -> (config, batch, image size, num_registers, keep raw outputs, autocast-bf16)
CASES = {
    "xxs_cf_b4": (synth.canonical("XXS"), 4, 224, 3, True, True),
    "xxs_tf_b2": (synth.canonical("XXS", conv_first=False), 2, 224, 3, True, False),
    "m_cf_b2": (synth.canonical("M"), 2, 224, 3, False, True),
    "xl_cf_b2": (synth.canonical("XL"), 2, 224, 3, False, True),
    "s_base": (dict(SMALL), 2, 112, 3, True, False),
    "s_simplehead": (dict(SMALL, simple_mlp_output=True), 2, 112, 3, False, False),
    "s_poolhead": (dict(SMALL, head_output_from_register=False), 2, 112, 3, False, False),
    "s_poolhead_bias": (dict(SMALL, head_output_from_register=False, output_head_bias=True), 2, 112, 3, False, False),
    "s_convemb": (dict(SMALL, conv_embedding=True, conv_embedding_kernel_size=5), 2, 112, 3, True, False),
    "s_slowatt": (dict(SMALL, fast_att=False), 2, 112, 3, False, False),
    "s_bias": (dict(SMALL, mixer_ffn_bias=True, mixer_deptwise_bias=True, output_head_bias=True), 2, 112, 3, False, False),
    "s_k3": (dict(SMALL, conv_kernel_size=3), 2, 112, 3, False, False),
    "s_k5": (dict(SMALL, conv_kernel_size=5), 2, 112, 3, False, False),
    "s_relu": (dict(SMALL, activation="relu"), 2, 112, 3, False, False),
    "s_tanh": (dict(SMALL, activation="tanh"), 2, 112, 3, False, False),
    "s_sigmoid": (dict(SMALL, activation="sigmoid"), 2, 112, 3, False, False),
    "s_leaky": (dict(SMALL, activation="leaky_relu"), 2, 112, 3, False, False),
    "s_selu": (dict(SMALL, activation="selu"), 2, 112, 3, False, False),
    "s_noqv": (dict(SMALL, normalize_qv=False), 2, 112, 3, False, False),
    "s_nreg0": (dict(SMALL), 2, 112, 0, False, False),
    "s_nreg4": (dict(SMALL), 2, 112, 4, False, False),
    "s_tf": (dict(SMALL, conv_first=False), 2, 112, 3, False, False),
    "s_p8_img64": (dict(SMALL, patch_size=8), 3, 64, 3, True, False),
    "s_p14": (dict(SMALL, patch_size=14), 2, 112, 3, False, False),
    "s_embact_gelu": (dict(SMALL, embedding_activation="gelu"), 2, 112, 3, False, False),
    "s_blk1_mix1": (dict(SMALL, num_blocks=1, conv_block_num=1), 1, 112, 3, False, False),
    "s_c96_h8": (dict(SMALL, embedding_dim=96, n_head=8), 2, 112, 3, False, False),
    "s_c256_h2": (dict(SMALL, embedding_dim=256, n_head=2), 2, 112, 3, False, False),
}

WSEED = 231424314  # the reference harness seed (model_train.py:61)
XSEED = 0


def main():
    ref_model, ref_layers, ref_tu = import_reference()
    torch.set_num_threads(8)
    manifest = {}
    for name, (cfg, B, img, nreg, raw, do_bf16) in CASES.items():
        torch.manual_seed(0)
        m = ref_model.MainModel.from_dict(**cfg)
        m.eval()
        sd = synth.synth_state_dict(m, WSEED)
        m.load_state_dict(sd)
        x = synth.synth_images(XSEED, B, img)
        with torch.no_grad():
            ref_out = m(x.clone(), num_registers=nreg, return_raw_outputs=True)
            o_out = orc.forward(x.clone(), sd, cfg, num_registers=nreg, return_raw_outputs=True)
        errs = [float((a - b).abs().max()) for a, b in zip(ref_out, o_out)]
        assert max(errs) <= 1e-5, (name, errs)
        rec = dict(logits=ref_out[0].numpy())
        if raw:
            rec["raw_x"] = ref_out[1].contiguous().numpy()
            rec["raw_reg"] = ref_out[2].contiguous().numpy()
        if do_bf16:
            with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16):
                yb = m(x.clone(), num_registers=nreg)
            rec["logits_autocast_bf16"] = yb.float().numpy()
        meta = dict(config=cfg, batch=B, image=img, num_registers=nreg, wseed=WSEED, xseed=XSEED,
                    weights_sha256=weights_digest(sd),
                    images_sha256=hashlib.sha256(x.numpy().tobytes()).hexdigest(),
                    oracle_vs_reference_maxabs=max(errs))
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), meta=json.dumps(meta), **rec)
        manifest[name] = meta
        bf = ""
        if do_bf16:
            bf = f" autocast-bf16 err {np.abs(rec['logits_autocast_bf16'] - rec['logits']).max():.2e}"
        print(f"{name}: logits std {rec['logits'].std():.4f} oracle err {max(errs):.1e}{bf}", flush=True)

    # ---- module-level fixtures ------------------------------------------------
    mod = {}
    g = torch.linspace(-6, 6, 2401)
    mod["kelu_x"] = g.numpy()
    mod["kelu_y"] = ref_tu.KeLu(g).numpy()
    assert float((orc.kelu(g) - ref_tu.KeLu(g)).abs().max()) <= 1e-6

    # channel LayerNorm (layers.py:12-24) on NCHW
    ln = ref_layers.LayerNorm(48)
    lsd = synth.synth_state_dict(ln, WSEED)
    ln.load_state_dict(lsd)
    xl = torch.from_numpy(synth.normal(77, 2 * 48 * 5 * 6).astype(np.float32).reshape(2, 48, 5, 6) * 3 + 1)
    mod["cln_x"] = xl.numpy()
    mod["cln_y"] = ln(xl).detach().numpy()

    # standalone ConvMixer (C=64, 8x8) and EncoderLayer with a mask on the manual path
    cm = ref_layers.ConvMixer(64, kernel_size=7, mixer_ffn_bias=True, mixer_deptwise_bias=True).eval()
    cm.load_state_dict(synth.synth_state_dict(cm, WSEED))
    xc = torch.from_numpy(synth.normal(78, 2 * 64 * 8 * 8).astype(np.float32).reshape(2, 64, 8, 8))
    with torch.no_grad():
        mod["mixer_x"] = xc.numpy()
        mod["mixer_y"] = cm(xc).numpy()

    enc = ref_layers.EncoderLayer(64, n_head=4, activation_func=ref_tu.KeLu, fast_att=False).eval()
    enc.load_state_dict(synth.synth_state_dict(enc, WSEED))
    xe = torch.from_numpy(synth.normal(79, 2 * 64 * 8 * 8).astype(np.float32).reshape(2, 64, 8, 8))
    re = torch.from_numpy(synth.normal(80, 2 * 4 * 64).astype(np.float32).reshape(2, 4, 64))
    with torch.no_grad():
        ye, rge = enc(xe, re)
    mod["enc_kelu_x"], mod["enc_kelu_reg"] = xe.numpy(), re.numpy()
    mod["enc_kelu_y"], mod["enc_kelu_yreg"] = ye.numpy(), rge.numpy()
    np.savez_compressed(os.path.join(HERE, "modules.npz"), **mod)

    # ---- module-tree / state_dict surface + RNG-order fidelity of construction ----
    surface = {}
    for sname, scfg in [("XXS", synth.canonical("XXS")), ("M", synth.canonical("M")),
                        ("XL", synth.canonical("XL")), ("s_convemb", CASES["s_convemb"][0]),
                        ("s_poolhead_bias", CASES["s_poolhead_bias"][0]), ("s_bias", CASES["s_bias"][0]),
                        ("defaults", {})]:
        torch.manual_seed(1234)
        m = ref_model.MainModel.from_dict(**scfg)
        sd = m.state_dict()
        surface[sname] = dict(config=scfg,
                              keys=[[k, list(v.shape), str(v.dtype)] for k, v in sd.items()],
                              init_sha256_seed1234=weights_digest(sd) if sname not in ("M", "XL") else None,
                              num_params=m.return_num_params())
    with open(os.path.join(HERE, "surface.json"), "w") as f:
        json.dump(surface, f)

    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("wrote", len(CASES), "model fixtures + modules.npz")


if __name__ == "__main__":
    main()
