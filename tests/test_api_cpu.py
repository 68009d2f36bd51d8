"""Drop-in API surface (no GPU): module tree / state-dict keys identical to the reference's
VapGPT(VapConfig()).state_dict(), strict loading, LSTM depth inference, config + CLI flags."""
import argparse

import numpy as np
import pytest
import torch

from voiceactivityprojection_amd.weights import schema, synthetic_state_dict


def test_imports_like_reference():
    from vap.model import BIN_TIMES, VAPModel, VapConfig, VapGPT, load_older_state_dict  # noqa: F401
    from vap.objective import ObjectiveVAP  # noqa: F401
    assert BIN_TIMES == [0.2, 0.4, 0.6, 0.8]
    assert issubclass(VAPModel, VapGPT)


def test_state_dict_schema_matches_reference_keys():
    from vap.model import VapGPT

    m = VapGPT()
    sd = m.state_dict()
    ref = dict(schema())
    assert set(sd) == set(ref)
    for k, shp in ref.items():
        assert tuple(sd[k].shape) == shp, k
    # codebook is the reference's fixed code vector table
    emb = sd["objective.codebook.emb.weight"].numpy()
    assert emb.shape == (256, 8) and (emb[5] == np.array([1, 0, 1, 0, 0, 0, 0, 0])).all()


def test_strict_load_and_unexpected_key():
    from vap.model import VapGPT

    m = VapGPT()
    sd = {k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0).items()}
    m.load_state_dict(sd, strict=True)
    bad = dict(sd)
    bad["foo.bar"] = torch.zeros(1)
    with pytest.raises(RuntimeError):
        m.load_state_dict(bad, strict=True)


def test_lstm_depth_inferred_from_state_dict():
    from vap.model import VapGPT

    m = VapGPT()
    sd2 = {k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0, lstm_layers=2).items()}
    m.load_state_dict(sd2, strict=True)
    assert m.lstm_layers == 2
    assert "encoder.encoder.gAR.baseNet.weight_hh_l1" in m.state_dict()


def test_config_argparse_roundtrip():
    from vap.model import VapConfig

    p = argparse.ArgumentParser()
    p, fields = VapConfig.add_argparse_args(p, [])
    args = p.parse_args(["--vap_cross_layers", "2", "--vap_bin_times", "0.2", "0.4", "0.6", "0.8"])
    conf = VapConfig.args_to_conf(args)
    assert conf.cross_layers == 2 and conf.bin_times == [0.2, 0.4, 0.6, 0.8] and conf.dim == 256
    assert set(fields) >= {"sample_rate", "frame_hz", "bin_times", "dim", "channel_layers", "cross_layers",
                           "num_heads", "dropout", "freeze_encoder", "load_pretrained"}


def test_model_properties():
    from vap.model import VapGPT

    m = VapGPT()
    assert m.horizon_time == pytest.approx(2.0)
    assert m.sample_rate == 16000 and m.frame_hz == 50
    assert m.objective.n_classes == 256 and m.objective.horizon == 100
    with pytest.raises(RuntimeError, match="no CPU fallback"):  # attention maps run on the engine too
        m(torch.zeros(1, 2, 40960), attention=True)


def test_codebook_encode_matches_bit_packing():
    from vap.objective import Codebook

    cb = Codebook([10, 20, 30, 40])
    x = torch.randint(0, 2, (50, 2, 4)).float()
    idx = cb.encode(x)
    exp = (x[:, 0] * torch.tensor([1, 2, 4, 8])).sum(-1) + (x[:, 1] * torch.tensor([16, 32, 64, 128])).sum(-1)
    assert torch.equal(idx, exp.long())
    assert torch.equal(cb.decode(idx), x)
