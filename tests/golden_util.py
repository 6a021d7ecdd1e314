"""Shared helpers to load golden fixtures and rebuild their inputs/weights."""
import json
import os

import numpy as np
import torch

import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_case(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    arrays = {k: z[k] for k in z.files if k != "meta"}
    return meta, arrays


def case_names():
    with open(os.path.join(GOLDEN, "MANIFEST.json")) as f:
        return sorted(json.load(f).keys())


def build_inputs(meta, model):
    """Synthetic state_dict for ``model`` and the case's images (CPU fp32)."""
    sd = synth.synth_state_dict(model, meta["wseed"])
    x = synth.synth_images(meta["xseed"], meta["batch"], meta["image"])
    return sd, x


def digest(sd):
    import hashlib
    h = hashlib.sha256()
    for k, v in sd.items():
        h.update(k.encode())
        h.update(v.detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()
