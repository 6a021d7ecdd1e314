"""CPU: the oracle against the golden fixtures made by the reference itself.

Pins (1) the portable weight/input generator (digests recorded when the goldens
were made), (2) that our module tree matches the reference's (the generator walks
OUR model here and must reproduce the reference-side weight digest), and (3) the
oracle's logits / raw outputs to <= 1e-5 of the reference's.
"""
import numpy as np
import pytest
import torch

import golden_util as gu
import sdpnet_oracle as orc
import synth

CASES = gu.case_names()


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference_golden(name):
    import model as ours
    meta, arr = gu.load_case(name)
    torch.manual_seed(0)
    m = ours.MainModel.from_dict(**meta["config"])
    sd, x = gu.build_inputs(meta, m)
    assert gu.digest(sd) == meta["weights_sha256"], "weight generator / module tree drifted"
    import hashlib
    assert hashlib.sha256(x.numpy().tobytes()).hexdigest() == meta["images_sha256"]
    out = orc.forward(x, sd, meta["config"], num_registers=meta["num_registers"], return_raw_outputs=True)
    np.testing.assert_allclose(out[0].numpy(), arr["logits"], atol=1e-5, rtol=0)
    if "raw_x" in arr:
        np.testing.assert_allclose(out[1].numpy(), arr["raw_x"], atol=1e-5, rtol=0)
        np.testing.assert_allclose(out[2].numpy(), arr["raw_reg"], atol=1e-5, rtol=0)


def test_oracle_kelu_grid():
    _, _ = None, None
    z = np.load(gu.GOLDEN + "/modules.npz")
    y = orc.kelu(torch.from_numpy(z["kelu_x"])).numpy()
    np.testing.assert_allclose(y, z["kelu_y"], atol=1e-6, rtol=0)


def test_oracle_channel_layernorm_fixture():
    z = np.load(gu.GOLDEN + "/modules.npz")
    from layers import LayerNorm
    ln = LayerNorm(48)
    sd = synth.synth_state_dict(ln, 231424314)
    y = orc.channel_layernorm(torch.from_numpy(z["cln_x"]), sd["gamma"], sd["beta"])
    np.testing.assert_allclose(y.numpy(), z["cln_y"], atol=1e-5, rtol=0)


def test_oracle_mixer_and_encoder_fixtures():
    z = np.load(gu.GOLDEN + "/modules.npz")
    from layers import ConvMixer, EncoderLayer
    from training_utilities import KeLu
    cm = ConvMixer(64, kernel_size=7, mixer_ffn_bias=True, mixer_deptwise_bias=True)
    sd = synth.synth_state_dict(cm, 231424314)
    y = orc.conv_mixer(torch.from_numpy(z["mixer_x"]), sd, "", "gelu")
    np.testing.assert_allclose(y.numpy(), z["mixer_y"], atol=1e-5, rtol=0)
    enc = EncoderLayer(64, n_head=4, activation_func=KeLu, fast_att=False)
    sd = synth.synth_state_dict(enc, 231424314)
    ye, re = orc.encoder_layer(torch.from_numpy(z["enc_kelu_x"]), torch.from_numpy(z["enc_kelu_reg"]), sd, "", 4,
                               "kelu", True, False)
    np.testing.assert_allclose(ye.numpy(), z["enc_kelu_y"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(re.numpy(), z["enc_kelu_yreg"], atol=1e-5, rtol=0)
