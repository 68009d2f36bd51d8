"""Pin the CPU oracle (oracle/vap_oracle.py) against golden vectors produced by the REFERENCE
implementation (tools/gen_golden.py). CPU only."""
import json
import os

import numpy as np
import pytest
import torch

import vap_oracle as O
from voiceactivityprojection_amd.weights import synthetic_state_dict, synthetic_waveform

TOL = 2e-5  # oracle vs reference: same ATen op sequence, fp32 (SURVEY.md §8(c) noise floor)


def _sd(layers=1):
    return O.state_dict_to_torch(synthetic_state_dict(seed=0, lstm_layers=layers))


def _check(out, g, keys=("vad", "p_now", "p_future", "H", "loss"), tol=TOL):
    for k in keys:
        np.testing.assert_allclose(out[k].numpy(), g[k], atol=tol, rtol=0, err_msg=k)


def test_frame_lengths_known_answers():
    # SURVEY.md §8(a) A1 verified values
    assert O.frame_lengths(320000)[-1] == 1000
    assert O.frame_lengths(37392)[-1] == 117
    assert O.frame_lengths(320319)[-1] == 1001
    assert O.frame_lengths(960000)[-1] == 3000
    assert O.frame_lengths(160000)[-1] == 500


def test_short_clip_stage_taps(golden):
    g = golden("short_clip")
    taps = {}
    out = O.probs(torch.from_numpy(g["waveform"]), _sd(), taps=taps)
    np.testing.assert_allclose(taps["lstm"][:, :64].numpy(), g["lstm1_head"], atol=TOL)
    np.testing.assert_allclose(taps["enc1"].numpy(), g["enc1"], atol=TOL)
    np.testing.assert_allclose(taps["enc2"].numpy(), g["enc2"], atol=TOL)
    np.testing.assert_allclose(taps["ar_channel1"].numpy(), g["ar_channel1"], atol=TOL)
    np.testing.assert_allclose(taps["logits"].numpy(), g["logits"], atol=5e-5)
    np.testing.assert_allclose(taps["vad_logits"].numpy(), g["vad_logits"], atol=5e-5)
    _check(out, g, keys=("probs", "vad", "p_now", "p_future", "H", "loss"))


def test_waveform_generator_matches_fixture(golden):
    g = golden("short_clip")
    np.testing.assert_array_equal(synthetic_waveform(int(g["clip_index"]), g["waveform"].shape[-1])[None], g["waveform"])
    g = golden("batch_20s")
    w = np.stack([synthetic_waveform(i, int(g["n_samples"])) for i in (0, 1)])
    np.testing.assert_array_equal(w[:, :, :16], g["wav_head"])
    np.testing.assert_allclose([w.astype(np.float64).sum(), (w.astype(np.float64) ** 2).sum()], g["wav_stats"], rtol=1e-12)


@pytest.mark.slow
def test_batch_20s(golden):
    g = golden("batch_20s")
    w = np.stack([synthetic_waveform(i, int(g["n_samples"])) for i in (0, 1)])
    out = O.probs(torch.from_numpy(w), _sd())
    _check(out, g)
    np.testing.assert_allclose(out["probs"][:, :8].numpy(), g["probs_head"], atol=TOL)


@pytest.mark.slow
def test_bench4_clip(golden):
    """The bench configuration's fixture (tools/gen_golden.py bench4): its inputs are the bench's own
    synthetic_batch, and the oracle reproduces the reference on one of its clips."""
    from voiceactivityprojection_amd.weights import synthetic_batch

    g = golden("bench4_20s")
    w = synthetic_batch(0, 4, int(g["n_samples"]))
    np.testing.assert_allclose([w.astype(np.float64).sum(), (w.astype(np.float64) ** 2).sum()], g["wav_stats"],
                               rtol=1e-12)
    out = O.probs(torch.from_numpy(w[2:3]), _sd())
    _check(out, {k: g[k][2:3] for k in ("vad", "p_now", "p_future", "H", "loss")})
    np.testing.assert_allclose(out["probs"][:, ::10].numpy(), g["probs_stride10"][2:3], atol=TOL)


def test_example_wav_loader_and_oracle(golden):
    """BASELINE configs[0]: the build's load_waveform on the reference's example wav gives the fixture's
    input (int16 / 32768, 24 -> 16 kHz, 37392 samples, zero second channel), and the oracle matches
    the reference's probs on it.  (The resampler itself is unpinned: torchaudio is absent.)"""
    from voiceactivityprojection_amd.audio import load_waveform

    g = golden("example_wav")
    x, sr = load_waveform(os.path.join(os.path.dirname(__file__), "golden", "student_long_female_en-US-Wavenet-G.wav"))
    assert sr == 16000 and tuple(x.shape) == (1, 37392)
    np.testing.assert_array_equal(x.numpy(), g["waveform"][0, :1])
    assert not g["waveform"][0, 1].any()
    out = O.probs(torch.from_numpy(g["waveform"]), _sd())
    _check(out, g, keys=("probs", "vad", "p_now", "p_future", "H", "loss"))


@pytest.mark.parametrize("name", ["len_37392", "len_min"])
def test_ragged_lengths(golden, name):
    g = golden(name)
    out = O.probs(torch.from_numpy(g["waveform"]), _sd())
    _check(out, g)


def test_too_short_raises():
    meta = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "meta.json")))
    with pytest.raises(RuntimeError):
        O.probs(torch.from_numpy(synthetic_waveform(14, 32000)[None]), _sd())
    assert "size is 100" in meta["short_clip_error"]


def test_lstm2_variant(golden):
    g = golden("lstm2_short")
    out = O.probs(torch.from_numpy(g["waveform"]), _sd(2))
    _check(out, g, keys=("probs", "vad", "p_now", "p_future", "H", "loss"))


def test_lstm_loop_matches_module():
    sd = _sd()
    x = torch.randn(2, 50, 256)
    np.testing.assert_allclose(O.lstm_loop(x, sd).numpy(), O.lstm(x, sd).numpy(), atol=2e-6)


def test_labels_bit_exact(golden):
    g = golden("labels_kat")
    n = len(g["names"])
    for i in range(n):
        va = g[f"va_{i}"][None]
        if va.shape[1] - 1 < 100:
            with pytest.raises(RuntimeError):
                O.get_labels_np(va, [10, 20, 30, 40])
            continue
        np.testing.assert_array_equal(O.get_labels_np(va, [10, 20, 30, 40]), g[f"labels_{i}"], err_msg=str(g["names"][i]))
    soft = g["soft_va"]
    ratios = O.label_ratios_np(soft, [10, 20, 30, 40])
    safe = (np.abs(ratios - 0.5) > 1e-6).all(axis=(-1, -2))
    got = O.get_labels_np(soft, [10, 20, 30, 40])
    np.testing.assert_array_equal(got[safe], g["soft_labels"][safe])
    assert safe.mean() > 0.95


def test_oracle_attention_maps_vs_reference(golden):
    """attention=True maps of the oracle against the reference's own (tools/gen_golden.py attention)."""
    g = golden("attention_maps")
    sd = _sd()
    out = O.forward(torch.from_numpy(g["waveform"]), sd, attention=True)
    for k in ("logits", "vad_logits", "self_attn", "cross_attn", "cross_self_attn"):
        ref = g[k]
        got = out["vad" if k == "vad_logits" else k].numpy()
        assert got.shape == ref.shape, (k, got.shape, ref.shape)
        err = float(np.abs(got - ref).max())
        assert err < 1e-5, f"{k}: {err}"


def test_oracle_mono_vs_reference(golden):
    """VapGPTMono forward (with va_history) and probs (without, as the reference's probs()) of the
    oracle against the reference's own outputs (tools/gen_golden.py mono)."""
    g = golden("mono")
    sd = O.state_dict_to_torch(synthetic_state_dict(seed=0, mono=True, va_history_bins=5))
    w, va, hist = (torch.from_numpy(g[k]) for k in ("waveform", "va", "va_history"))
    out = O.forward_mono(w, va, sd, hist)
    assert float((out["logits"] - torch.from_numpy(g["logits"])).abs().max()) < 1e-4
    pr = O.probs_mono(w, va, sd)
    for k, gk in (("probs", "probs_logits_nohist"), ("p_now", "p_now"), ("p_future", "p_future"), ("H", "H")):
        assert float((pr[k] - torch.from_numpy(g[gk])).abs().max()) < 2e-5, k
