"""GPU parity: the HIP engine (through the C ABI) vs golden vectors from the REFERENCE and vs the
CPU oracle on identical inputs.

Tolerances (stated per north_star "within a stated fp tolerance"):
  * fp32 parity mode: 1e-4 absolute on probs / vad / p_now / p_future, 1e-3 on H and loss
    (H and the CE loss sum / log 256 terms; observed error is ~1e-6).
  * bf16 perf mode: BF16_TOL below (bf16 storage of activations and weights, fp32 accumulate).
  * labels: bit-exact (integer).
"""
import numpy as np
import pytest
import torch

import vap_oracle as O
from voiceactivityprojection_amd.weights import synthetic_state_dict, synthetic_waveform

pytestmark = pytest.mark.gpu

# the stated tolerances (voiceactivityprojection_amd/tolerances.py): fp32 1e-4 / 1e-3; bf16 <= 3x the largest
# error measured against the reference fixtures (tools/bf16_errors.py, profiles/r3_bf16_errors_s2.json:
# probs 1.42e-3, vad 1.34e-2, p_now 5.5e-4, p_future 4.8e-4, H 8.9e-3, loss 1.61e-2 over short_clip,
# example_wav, len_*, batch_20s, bench4_20s, long_60s)
from voiceactivityprojection_amd.tolerances import BF16_TOL, FP32_TOL  # noqa: E402


def _model(precision="fp32", lstm_layers=1):
    from vap.model import VapGPT

    m = VapGPT(precision=precision, lstm_layers=lstm_layers)
    sd = {k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0, lstm_layers=lstm_layers).items()}
    m.load_state_dict(sd, strict=True)
    return m.to("cuda").eval()


@pytest.fixture(scope="module")
def m32():
    return _model("fp32")


@pytest.fixture(scope="module")
def m16():
    return _model("bf16")


def _cmp(out, ref, tol, keys=("vad", "p_now", "p_future", "H", "loss")):
    errs = {}
    for k in keys:
        got = out[k].float().cpu().numpy()
        exp = ref[k]
        assert got.shape == exp.shape, (k, got.shape, exp.shape)
        errs[k] = float(np.abs(got - exp).max())
    bad = {k: e for k, e in errs.items() if not e <= tol[k]}
    assert not bad, f"tolerance exceeded: {bad} (all: {errs})"
    return errs


def test_short_clip_fp32(m32, golden):
    g = golden("short_clip")
    w = torch.from_numpy(g["waveform"]).cuda()
    out = m32.probs(w)
    _cmp(out, g, FP32_TOL, keys=("probs", "vad", "p_now", "p_future", "H", "loss"))
    x1, x2 = m32.encode_audio(w)
    np.testing.assert_allclose(x1.cpu().numpy(), g["enc1"], atol=1e-4)
    np.testing.assert_allclose(x2.cpu().numpy(), g["enc2"], atol=1e-4)
    fw = m32(w)
    np.testing.assert_allclose(fw["logits"].cpu().numpy(), g["logits"], atol=5e-4)
    np.testing.assert_allclose(fw["vad"].cpu().numpy(), g["vad_logits"], atol=5e-4)


def test_batch_20s_fp32(m32, golden):
    g = golden("batch_20s")
    w = np.stack([synthetic_waveform(i, int(g["n_samples"])) for i in (0, 1)])
    out = m32.probs(torch.from_numpy(w).cuda())
    _cmp(out, g, FP32_TOL)
    np.testing.assert_allclose(out["probs"][:, :8].cpu().numpy(), g["probs_head"], atol=1e-4)
    np.testing.assert_allclose(out["probs"][:, -8:].cpu().numpy(), g["probs_tail"], atol=1e-4)


def test_long_60s_fp32(m32, golden):
    g = golden("long_60s")
    w = synthetic_waveform(int(g["clip_start"]), int(g["n_samples"]))[None]
    out = m32.probs(torch.from_numpy(w).cuda())
    _cmp(out, g, FP32_TOL)


@pytest.mark.parametrize("name", ["len_37392", "len_min"])
def test_ragged_fp32(m32, golden, name):
    g = golden(name)
    out = m32.probs(torch.from_numpy(g["waveform"]).cuda())
    _cmp(out, g, FP32_TOL)


def test_len_320319_fp32(m32, golden):
    g = golden("len_320319")
    w = synthetic_waveform(int(g["clip_start"]), int(g["n_samples"]))[None]
    out = m32.probs(torch.from_numpy(w).cuda())
    _cmp(out, g, FP32_TOL)


def test_too_short_raises(m32):
    w = torch.from_numpy(synthetic_waveform(14, 32000)[None]).cuda()
    with pytest.raises(RuntimeError, match="size is 100"):
        m32.probs(w)


def test_bad_channels_assert(m32):
    with pytest.raises(AssertionError):
        m32(torch.zeros(1, 1, 40960, device="cuda"))


def test_lstm2_fp32(golden):
    g = golden("lstm2_short")
    m = _model("fp32", lstm_layers=2)
    out = m.probs(torch.from_numpy(g["waveform"]).cuda())
    _cmp(out, g, FP32_TOL, keys=("probs", "vad", "p_now", "p_future", "H", "loss"))


def test_batch_invariance_and_determinism(m32):
    n = 40960
    w = torch.from_numpy(np.stack([synthetic_waveform(i, n) for i in range(3)])).cuda()
    a = m32.probs(w)
    b = m32.probs(w)
    c = m32.probs(w[1:2])
    for k in a:
        assert torch.equal(a[k], b[k]), f"run-to-run difference in {k}"
        assert torch.equal(a[k][1:2], c[k]), f"batch dependence in {k}"


def test_vs_oracle_random_batch(m32, sd_np):
    n = 48000
    w = np.stack([synthetic_waveform(50 + i, n) for i in range(3)])
    ref = O.probs(torch.from_numpy(w), O.state_dict_to_torch(sd_np))
    out = m32.probs(torch.from_numpy(w).cuda())
    _cmp(out, {k: v.numpy() for k, v in ref.items()}, FP32_TOL, keys=("probs", "vad", "p_now", "p_future", "H", "loss"))


def test_labels_bit_exact(m32, golden):
    g = golden("labels_kat")
    for i in range(len(g["names"])):
        va = torch.from_numpy(g[f"va_{i}"][None]).cuda()
        if va.shape[1] - 1 < 100:
            with pytest.raises(RuntimeError):
                m32.objective.get_labels(va)
            continue
        got = m32.objective.get_labels(va).cpu().numpy()
        np.testing.assert_array_equal(got, g[f"labels_{i}"], err_msg=str(g["names"][i]))
    soft = g["soft_va"]
    ratios = O.label_ratios_np(soft, [10, 20, 30, 40])
    safe = (np.abs(ratios - 0.5) > 1e-6).all(axis=(-1, -2))
    got = m32.objective.get_labels(torch.from_numpy(soft).cuda()).cpu().numpy()
    np.testing.assert_array_equal(got[safe], g["soft_labels"][safe])


def test_aggregate_and_vad_post(m32):
    torch.manual_seed(0)
    logits = torch.randn(2, 130, 256) * 3
    probs = logits.softmax(-1)
    got = m32.objective.probs_next_speaker_aggregate(probs.cuda(), 0, 1).cpu()
    exp = O.probs_next_speaker_aggregate(probs, 0, 1)
    np.testing.assert_allclose(got.numpy(), exp.numpy(), atol=1e-6)
    # VapGPT.vad post-processing vs the reference utilities (host loop semantics)
    from voiceactivityprojection_amd.utils import vad_fill_silences, vad_omit_spikes
    w = torch.from_numpy(np.stack([synthetic_waveform(70 + i, 40960) for i in range(2)])).cuda()
    for fill, omit in ((0.02, 0.02), (0.1, 0.04), (0.2, 0.2)):
        got = m32.vad(w, max_fill_silence_time=fill, max_omit_spike_time=omit).cpu()
        vl = m32(w)["vad"].cpu()
        exp = (vl.sigmoid() >= 0.5).float()
        for b in range(exp.shape[0]):
            exp[b] = vad_fill_silences(exp[b], max_fill_time=fill, frame_hz=50)
            exp[b] = vad_omit_spikes(exp[b], max_omit_time=omit, frame_hz=50)
        assert torch.equal(got, exp)


def test_short_clip_bf16(m16, golden):
    g = golden("short_clip")
    out = m16.probs(torch.from_numpy(g["waveform"]).cuda())
    errs = _cmp(out, g, BF16_TOL, keys=("probs", "vad", "p_now", "p_future", "H", "loss"))
    print("bf16 short clip max abs err:", errs)


def test_batch_20s_bf16(m16, golden):
    g = golden("batch_20s")
    w = np.stack([synthetic_waveform(i, int(g["n_samples"])) for i in (0, 1)])
    out = m16.probs(torch.from_numpy(w).cuda())
    errs = _cmp(out, g, BF16_TOL)
    for k, sl in (("probs_head", slice(0, 8)), ("probs_tail", slice(-8, None))):
        e = float((out["probs"][:, sl].cpu() - torch.from_numpy(g[k])).abs().max())
        assert e <= BF16_TOL["probs"], (k, e)
    print("bf16 20 s max abs err:", errs)


@pytest.mark.parametrize("name", ["len_37392", "len_min", "len_320319"])
def test_ragged_bf16(m16, golden, name):
    """Ragged lengths (T = 117, the minimum 101, 1001) in the bf16 perf path against the reference."""
    g = golden(name)
    w = g["waveform"] if "waveform" in g else synthetic_waveform(int(g["clip_start"]), int(g["n_samples"]))[None]
    out = m16.probs(torch.from_numpy(w).cuda())
    errs = _cmp(out, g, BF16_TOL)
    e = float((out["probs"][:, -4:].cpu() - torch.from_numpy(g["probs_tail"])).abs().max())
    assert e <= BF16_TOL["probs"], ("probs", e)
    print(f"bf16 {name} max abs err:", dict(errs, probs=e))


def test_bf16_multi_workgroup_batch_invariance(m16, m32):
    """B = 9 -> 18 sequences -> two LSTM workgroups (16 sequences each) in bf16 mode: every clip's
    outputs must be bit-identical to running that clip alone, and close to fp32 parity mode."""
    n = 40960
    w = torch.from_numpy(np.stack([synthetic_waveform(200 + i, n) for i in range(9)])).cuda()
    full = m16.probs(w)
    ref = m32.probs(w)
    for i in (0, 8):
        one = m16.probs(w[i:i + 1])
        for k in full:
            assert torch.equal(full[k][i:i + 1], one[k]), f"bf16 batch dependence in {k} (clip {i})"
    for k in ("p_now", "p_future", "vad"):
        err = (full[k] - ref[k]).abs().max().item()
        assert err <= BF16_TOL[k], (k, err)


def test_encoder_bf16_vs_reference(m16, golden):
    """bf16 encoder (fused conv0->conv1, resident LSTM) against the reference's EncoderCPC taps."""
    g = golden("short_clip")
    x1, x2 = m16.encode_audio(torch.from_numpy(g["waveform"]).cuda())
    for got, exp in ((x1, g["enc1"]), (x2, g["enc2"])):
        err = (got.cpu().numpy() - exp).__abs__().max()
        print("bf16 encoder max abs err:", err)
        assert err < 0.06, f"bf16 encoder max abs err {err}"  # <= 3x the measured 2.12e-2 (r4s2)


def test_long_60s_bf16(m16, golden):
    """BASELINE configs[3] clip length (60 s, T = 3000) through the bf16 time-pipelined path."""
    g = golden("long_60s")
    w = synthetic_waveform(int(g["clip_start"]), int(g["n_samples"]))[None]
    out = m16.probs(torch.from_numpy(w).cuda())
    errs = _cmp(out, g, BF16_TOL)
    e = float((out["probs"][:, -4:].cpu() - torch.from_numpy(g["probs_tail"])).abs().max())
    assert e <= BF16_TOL["probs"], ("probs", e)
    print("bf16 60 s max abs err:", dict(errs, probs=e))


def _bench4(g):
    from voiceactivityprojection_amd.weights import synthetic_batch

    return synthetic_batch(0, 4, int(g["n_samples"]))


def test_bench4_fp32_vs_reference(m32, golden):
    """The bench configuration's clips (20 s, the bench's own synthetic_batch clips 0..3) in parity
    mode against the reference's outputs: every frame of every per-frame output, probs on every
    10th frame."""
    g = golden("bench4_20s")
    out = m32.probs(torch.from_numpy(_bench4(g)).cuda())
    m32.synchronize()
    _cmp(out, g, FP32_TOL)
    np.testing.assert_allclose(out["probs"][:, ::10].cpu().numpy(), g["probs_stride10"], atol=FP32_TOL["probs"])


def test_bench_shape_bf16(m16, golden):
    """The bench workload itself (BASELINE configs[1]: 64 x 20 s, bf16, the time-pipelined schedule)
    checked against the REFERENCE: clips 0..3 of the bench batch are the bench4_20s fixture's clips
    (every per-frame output, probs on every 10th frame, within BF16_TOL); sampled clips are
    bit-identical to the same clip run alone (the schedule does not leak across clips); every output
    is finite."""
    from voiceactivityprojection_amd.weights import synthetic_batch

    g = golden("bench4_20s")
    w = torch.from_numpy(synthetic_batch(0, 64, 320000)).cuda()
    full = m16.probs(w)
    m16.synchronize()
    assert full["probs"].shape == (64, 1000, 256)
    head = {k: v[:4] for k, v in full.items()}
    errs = _cmp(head, g, BF16_TOL)
    e = float((head["probs"][:, ::10].cpu() - torch.from_numpy(g["probs_stride10"])).abs().max())
    assert e <= BF16_TOL["probs"], ("probs", e)
    print("bf16 bench4 max abs err:", dict(errs, probs=e))
    for i in (0, 37, 63):
        one = m16.probs(w[i:i + 1])
        for k in full:
            assert torch.equal(full[k][i:i + 1], one[k]), f"bf16 batch dependence in {k} (clip {i})"
    for k in ("probs", "p_now", "p_future", "vad", "H", "loss"):
        assert torch.isfinite(full[k]).all(), k


def test_long_60s_batch32_bf16(m16, golden):
    """BASELINE configs[3] at its configured size: 32 x 60 s (T = 3000, AliBi extrapolation past the
    20 s training length) through the bf16 time-pipelined schedule with a full batch.  The reference's
    60 s clip (seed 7) sits at batch index 5 and must match long_60s.npz within BF16_TOL; sampled
    clips are bit-identical to the same clip alone; every output is finite."""
    from voiceactivityprojection_amd.weights import synthetic_batch

    g = golden("long_60s")
    n = int(g["n_samples"])
    w = synthetic_batch(1000, 32, n)
    w[5] = synthetic_waveform(int(g["clip_start"]), n)
    w = torch.from_numpy(w).cuda()
    full = m16.probs(w)
    m16.synchronize()
    assert full["probs"].shape == (32, 3000, 256) and full["loss"].shape == (32, 2900)
    errs = _cmp({k: v[5:6] for k, v in full.items()}, g, BF16_TOL)
    e = float((full["probs"][5:6, -4:].cpu() - torch.from_numpy(g["probs_tail"])).abs().max())
    assert e <= BF16_TOL["probs"], ("probs", e)
    print("bf16 60 s @ batch 32 max abs err:", dict(errs, probs=e))
    for i in (0, 5, 31):
        one = m16.probs(w[i:i + 1])
        for k in full:
            assert torch.equal(full[k][i:i + 1], one[k]), f"bf16 batch dependence in {k} (clip {i})"
    for k in ("probs", "p_now", "p_future", "vad", "H", "loss"):
        assert torch.isfinite(full[k]).all(), k


ATTN_KEYS = ("self_attn", "cross_attn", "cross_self_attn")


def test_attention_maps_fp32_vs_reference(m32, golden):
    """forward(attention=True) (model.py:249-268): every layer's softmax weights against the
    reference's own maps (tests/golden/attention_maps.npz), fp32 mode, 1e-4 absolute."""
    g = golden("attention_maps")
    w = torch.from_numpy(g["waveform"]).cuda()
    out = m32(w, attention=True)
    for k in ("logits",) + ATTN_KEYS:
        got = out[k].cpu().numpy()
        assert got.shape == g[k].shape, (k, got.shape, g[k].shape)
        err = float(np.abs(got - g[k]).max())
        assert err < 1e-4, f"{k}: {err}"
    np.testing.assert_allclose(out["vad"].cpu().numpy(), g["vad_logits"], atol=1e-4)
    # rows are distributions over the causal past; the plain forward gives the same logits
    sa = out["self_attn"]
    assert torch.allclose(sa.sum(-1), torch.ones_like(sa.sum(-1)), atol=1e-5)
    assert float(torch.triu(sa, diagonal=1).abs().max()) == 0.0
    plain = m32(w)
    assert torch.equal(plain["logits"], out["logits"])


def test_attention_maps_bf16_vs_oracle(m16):
    """bf16 mode maps on a 2-clip batch against the oracle (fp32) on the same input."""
    wav = np.stack([synthetic_waveform(i, 16000) for i in (30, 31)])
    out = m16(torch.from_numpy(wav).cuda(), attention=True)
    ref = O.forward(torch.from_numpy(wav), O.state_dict_to_torch(synthetic_state_dict(seed=0)), attention=True)
    for k in ATTN_KEYS:
        got = out[k].cpu().numpy()
        exp = ref[k].numpy()
        assert got.shape == exp.shape, (k, got.shape, exp.shape)
        err = float(np.abs(got - exp).max())
        print(f"bf16 attention map {k} max abs err:", err)
        assert err < 1.9e-2, f"{k}: {err}"  # <= 3x the largest measured (cross_attn 6.3e-3, r4s2)


@pytest.mark.parametrize("B,T", [(3, 130), (2, 1000), (1, 101)])
def test_probs_loss_fused_equals_two_calls(m32, B, T):
    """vap_probs_loss (VapGPT.probs' epilogue: labels through LDS from the VAD logits, loss inside the
    softmax pass) is bit-identical to vap_probs followed by vap_labels_loss on vap_probs' vad."""
    import ctypes

    from voiceactivityprojection_amd import _native as N

    g = torch.Generator().manual_seed(B * 1000 + T)
    logits = (torch.randn(B, T, 256, generator=g) * 3).cuda()
    vadl = (torch.randn(B, T, 2, generator=g) * 2).cuda()
    obj = m32.objective
    n = T - obj.horizon
    bf = (ctypes.c_int * 4)(*obj.bin_frames)
    st = N.stream_ptr(logits.device)
    outs = []
    for fused in (False, True):
        o = {k: torch.empty(B, T, 256 if k == "probs" else 2, device="cuda") for k in ("probs", "vad", "p_now", "p_future")}
        o["H"] = torch.empty(B, T, device="cuda")
        o["labels"] = torch.empty(B, n, dtype=torch.int64, device="cuda")
        o["loss"] = torch.empty(B, n, device="cuda")
        ptrs = [o[k].data_ptr() for k in ("probs", "vad", "p_now", "p_future", "H")]
        if fused:
            N.check(N.lib().vap_probs_loss(logits.data_ptr(), vadl.data_ptr(), B, T, 4, 0, 1, 2, 3, bf, 0.5, *ptrs,
                                           o["labels"].data_ptr(), o["loss"].data_ptr(), st), "vap_probs_loss")
        else:
            N.check(N.lib().vap_probs(logits.data_ptr(), vadl.data_ptr(), B, T, 4, 0, 1, 2, 3, *ptrs, st), "vap_probs")
            N.check(N.lib().vap_labels_loss(logits.data_ptr(), o["vad"].data_ptr(), B, T, bf, 4, 0.5,
                                            o["labels"].data_ptr(), o["loss"].data_ptr(), st), "vap_labels_loss")
        torch.cuda.synchronize()
        outs.append({k: v.cpu() for k, v in o.items()})
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k


def test_vad_post_kernel_vs_reference_fixture(golden):
    """vad_post_kernel (VapGPT.vad's post-processing, vap/model.py:227-247) against the reference's own
    vad_fill_silences -> vad_omit_spikes outputs (tests/golden/vad_utils.npz): bit-exact."""
    from voiceactivityprojection_amd import _native as N

    g = golden("vad_utils")
    for i in range(4):
        va = torch.from_numpy(g[f"va_{i}"])
        logits = ((va * 2 - 1) * 10).contiguous().cuda()[None]  # sigmoid >= 0.5 exactly where va == 1
        T = va.shape[0]
        for fill, omit in ((0.02, 0.02), (0.06, 0.1), (0.2, 0.04)):
            out = torch.empty_like(logits)
            N.check(N.lib().vap_vad_postprocess(logits.data_ptr(), 1, T, 0.5, round(fill * 50), round(omit * 50),
                                                out.data_ptr(), N.stream_ptr(logits.device)), "vap_vad_postprocess")
            np.testing.assert_array_equal(out[0].cpu().numpy(), g[f"post_{i}_{fill}_{omit}"], err_msg=f"{i} {fill} {omit}")
