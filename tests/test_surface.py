"""CPU: the drop-in Python surface matches the reference's (module tree,
state_dict keys/shapes/dtypes, constructor kwargs, RNG-order of construction,
SdPModel utilities).  Reference facts come from tests/golden/surface.json,
recorded from the reference itself by gen_golden.py."""
import inspect
import json
import os

import pytest
import torch

import golden_util as gu
import sdpnet_oracle as orc

with open(os.path.join(gu.GOLDEN, "surface.json")) as f:
    SURFACE = json.load(f)


@pytest.mark.parametrize("name", sorted(SURFACE))
def test_state_dict_surface(name):
    import model as ours
    rec = SURFACE[name]
    torch.manual_seed(1234)
    m = ours.MainModel.from_dict(**rec["config"])
    sd = m.state_dict()
    got = [[k, list(v.shape), str(v.dtype)] for k, v in sd.items()]
    assert got == rec["keys"]
    assert m.return_num_params() == rec["num_params"]
    if rec["init_sha256_seed1234"] is not None:
        # same construction order => bit-identical initial parameters
        assert gu.digest(sd) == rec["init_sha256_seed1234"]
    assert m.config == rec["config"]


def test_constructor_kwargs_match_reference():
    import model as ours
    sig = inspect.signature(ours.MainModel.__init__)
    params = {k: v.default for k, v in sig.parameters.items() if k != "self"}
    assert params == orc.MAINMODEL_DEFAULTS  # restates model.py:28-54


def test_forward_signatures():
    import model as ours
    import layers as L
    f = inspect.signature(ours.MainModel.forward)
    assert list(f.parameters) == ["self", "x", "num_registers", "return_raw_outputs"]
    assert f.parameters["num_registers"].default == 3
    assert inspect.signature(L.EmbeddingLayer.forward).parameters["num_registers"].default == 0
    assert inspect.signature(L.ConvEmbedding.forward).parameters["num_registers"].default == 3
    for cls in (L.Block, L.EncoderLayer, L.FinalBlock):
        assert list(inspect.signature(cls.forward).parameters) == ["self", "x", "register", "mask"]


def test_kelu_activation_string_raises_like_reference():
    import model as ours
    # The reference puts the bare KeLu function into nn.Sequential (layers.py:83-92).
    with pytest.raises(TypeError):
        ours.MainModel(embedding_dim=32, num_blocks=1, n_head=2, activation="kelu")


def test_save_and_from_pretrained_roundtrip(tmp_path):
    import model as ours
    cfg = dict(embedding_dim=32, num_blocks=1, n_head=2, max_image_size=[16, 16])
    m = ours.MainModel.from_dict(**cfg)
    fn = str(tmp_path / "m")
    m.save_model(fn)
    m2 = ours.MainModel.from_pretrained(fn + ".pt")
    assert m2.config == cfg
    for (k, a), (k2, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert k == k2 and torch.equal(a, b)


def test_no_wandb_import():
    import sys
    import model  # noqa: F401
    import training_utilities  # noqa: F401
    assert "wandb" not in sys.modules


def test_cpu_forward_fails_loudly():
    import model as ours
    m = ours.MainModel(embedding_dim=32, num_blocks=1, n_head=2).eval()
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m(torch.randn(1, 3, 64, 64))


def test_train_mode_forward_has_no_cpu_fallback():
    """Train mode runs the HIP training path (sdpnet_train.py); on CPU tensors it raises
    instead of falling back to ATen."""
    import model as ours
    m = ours.MainModel(embedding_dim=32, num_blocks=1, n_head=2)
    assert m.training
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m(torch.randn(1, 3, 64, 64))
