"""Host-side plumbing (no GPU): run.py chunking + JSON contract, audio loading/resampling, VAD utils."""
import json
import os

import numpy as np
import pytest
import torch

import vap_oracle as O
from voiceactivityprojection_amd.weights import synthetic_state_dict, synthetic_waveform

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class OracleModel:
    """CPU stand-in for VapGPT in host-logic tests (the oracle is the checker, not the product)."""

    sample_rate, frame_hz = 16000, 50

    def __init__(self):
        self.sd = O.state_dict_to_torch(synthetic_state_dict(seed=0))

    def probs(self, w):
        return O.probs(w, self.sd)

    def synchronize(self):
        self.synced = True


def test_step_extraction_matches_per_fold_reference_loop():
    import run

    m = OracleModel()
    n = 16000 * 13 + 1234  # 13.08 s: several folds + tail
    w = torch.from_numpy(np.stack([synthetic_waveform(300, n)]))
    got = run.step_extraction(w, m, "cpu", context_time=3, step_time=2, fold_batch=3)
    # reference semantics (run.py:23-131), one fold at a time
    sr, fh = 16000, 50
    chunk, step = 5 * sr, 2 * sr
    folds = w.unfold(-1, chunk, step).permute(2, 0, 1, 3)
    exp = m.probs(folds[0])
    for f in folds[1:]:
        o = m.probs(f)
        for k in run.OUT_KEYS:
            exp[k] = torch.cat([exp[k], o[k][:, -2 * fh:]], 1)
    expected_frames = round(round(n / sr, 2) * fh)
    om = expected_frames - exp["p_now"].shape[1]
    if om:
        o = m.probs(w[..., -chunk:])
        for k in run.OUT_KEYS:
            exp[k] = torch.cat([exp[k], o[k][:, -om:]], 1)
    for k in run.OUT_KEYS + ("loss",):  # "loss" stays the first fold's (reference run.py:66)
        assert got[k].shape == exp[k].shape, k
        torch.testing.assert_close(got[k], exp[k], atol=1e-5, rtol=1e-5)  # CPU batch-size noise of the oracle
    assert set(got) == set(exp)
    assert got["p_now"].shape[1] == expected_frames


def test_json_contract(tmp_path):
    from voiceactivityprojection_amd.utils import tensor_dict_to_json, write_json

    out = {"probs": torch.rand(1, 3, 4), "vad": torch.rand(1, 3, 2), "H": torch.rand(1, 3)}
    f = tmp_path / "x.json"
    write_json(tensor_dict_to_json(out), str(f))
    d = json.load(open(f))
    assert set(d) == set(out) and np.allclose(np.array(d["probs"]), out["probs"].numpy())


def test_run_cli_args():
    import run

    args, conf = run.get_args(["-a", "x.wav", "--vap_cross_layers", "3", "-sd", "synthetic"])
    assert args.audio == "x.wav" and conf.cross_layers == 3 and args.state_dict == "synthetic"
    assert args.chunk_time == 30 and args.step_time == 5


def test_load_waveform_wav_roundtrip(tmp_path):
    from scipy.io import wavfile

    from voiceactivityprojection_amd.audio import load_waveform

    x = (np.sin(np.arange(16000) / 7.0) * 12000).astype(np.int16)
    p = tmp_path / "a.wav"
    wavfile.write(str(p), 16000, x)
    w, sr = load_waveform(str(p))
    assert sr == 16000 and w.shape == (1, 16000)
    np.testing.assert_allclose(w[0].numpy(), x / 32768.0, atol=1e-7)


def test_resample_properties():
    from voiceactivityprojection_amd.audio import resample

    # the example wav is 24 kHz, 56088 samples -> 37392 at 16 kHz
    x = torch.randn(1, 56088)
    y = resample(x, 24000, 16000)
    assert y.shape == (1, 37392)
    # a low-frequency tone survives resampling (parity with torchaudio is unpinned: SURVEY.md H6)
    t = torch.arange(24000) / 24000.0
    tone = torch.sin(2 * np.pi * 440 * t)[None]
    r = resample(tone, 24000, 16000)
    ref = torch.sin(2 * np.pi * 440 * torch.arange(16000) / 16000.0)
    assert (r[0, 200:-200] - ref[200:-200]).abs().max() < 2e-3


def test_example_wav_loads():
    p = "/root/reference/example/student_long_female_en-US-Wavenet-G.wav"
    if not os.path.exists(p):
        pytest.skip("reference example not present")
    from voiceactivityprojection_amd.audio import load_waveform

    w, sr = load_waveform(p, 16000)
    assert sr == 16000 and w.shape == (1, 37392)


def test_vad_utils_match_reference_semantics():
    from voiceactivityprojection_amd.utils import find_island_idx_len, vad_fill_silences, vad_omit_spikes

    x = torch.tensor([0, 0, 1, 1, 1, 0, 1, 0, 0, 0]).float()
    idx, dur, val = find_island_idx_len(x)
    assert idx.tolist() == [0, 2, 5, 6, 7] and dur.tolist() == [2, 3, 1, 1, 3] and val.tolist() == [0, 1, 0, 1, 0]
    v = torch.stack([x, 1 - x], -1)
    f = vad_fill_silences(v.clone(), max_fill_time=0.02, frame_hz=50)
    assert f[:, 0].tolist() == [0, 0, 1, 1, 1, 1, 1, 0, 0, 0]
    o = vad_omit_spikes(v.clone(), max_omit_time=0.02, frame_hz=50)
    assert o[:, 0].tolist() == [0, 0, 1, 1, 1, 0, 0, 0, 0, 0]


def test_vad_utils_vs_reference_fixture(golden):
    """The build's VAD helpers against the reference's own (tools/gen_golden.py utils, vap/utils.py):
    run lengths, fill-silence-then-omit-spike at several limits, onehot -> list -> onehot."""
    from voiceactivityprojection_amd.utils import (find_island_idx_len, vad_fill_silences, vad_list_to_onehot,
                                                   vad_omit_spikes, vad_onehot_to_vad_list)

    g = golden("vad_utils")
    for i in range(4):
        va = torch.from_numpy(g[f"va_{i}"])
        idx, dur, val = find_island_idx_len(va[:, 0])
        np.testing.assert_array_equal(np.stack([idx.numpy(), dur.numpy(), val.numpy().astype(np.int64)]),
                                      g[f"island_{i}"])
        for fill, omit in ((0.02, 0.02), (0.06, 0.1), (0.2, 0.04)):
            v = vad_omit_spikes(vad_fill_silences(va.clone(), max_fill_time=fill, frame_hz=50),
                                max_omit_time=omit, frame_hz=50)
            np.testing.assert_array_equal(v.numpy(), g[f"post_{i}_{fill}_{omit}"], err_msg=f"{i} {fill} {omit}")
        lists = vad_onehot_to_vad_list(va[None], frame_hz=50, ipu_thresh_time=0.1)
        assert lists == json.loads(str(g[f"list_{i}"])), i
        np.testing.assert_array_equal(vad_list_to_onehot(lists[0], duration=va.shape[0] / 50, frame_hz=50).numpy(),
                                      g[f"onehot_{i}"])
