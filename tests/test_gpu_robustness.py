"""Robustness of the persistent LSTM hand-off (bf16 path) at and beyond its CU budget, and error
reporting when a hand-off wait times out.

The time-pipelined forward runs ONE persistent recurrence launch whose workgroups (16 sequences
each, a whole CU: W_hh resident in LDS + registers) spin on ready flags that the caller stream's
conv kernels publish.  A launch that took every CU would leave the producers nowhere to run, so the
engine caps the persistent launch at half the CUs (VAP_LSTM_MAX_WG overrides) and runs a larger
batch through the same schedule in slices that fit.  Outputs must not depend on the slicing: every
clip stays bit-identical to the same clip run alone.
"""
import numpy as np
import pytest
import torch

from voiceactivityprojection_amd.weights import synthetic_state_dict, synthetic_waveform

pytestmark = pytest.mark.gpu



def _model(precision="bf16"):
    from vap.model import VapGPT

    m = VapGPT(precision=precision)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0).items()}, strict=True)
    return m.to("cuda").eval()


def _batch(B, n, seed):
    return torch.from_numpy(np.stack([synthetic_waveform(seed + i, n) for i in range(B)])).cuda()


def _same_as_alone(m, w, full, idx):
    for i in idx:
        one = m.probs(w[i:i + 1])
        for k in full:
            assert torch.equal(full[k][i:i + 1], one[k]), f"batch dependence in {k} (clip {i})"


def test_batch_above_persistent_cap_small(monkeypatch):
    """VAP_LSTM_MAX_WG=2: one pair of workgroups (16 sequences) per persistent launch, so a 20-clip
    batch runs as three slices and still matches every clip run alone."""
    monkeypatch.setenv("VAP_LSTM_MAX_WG", "2")
    m = _model()
    w = _batch(20, 40960, 700)
    full = m.probs(w)
    m.synchronize()
    _same_as_alone(m, w, full, (0, 7, 19))


def test_batch_at_and_above_default_cap():
    """Real sizes around the default cap (half of the CUs: 128 workgroups = 64 pairs = 512 stereo
    clips on a 256-CU MI355X): 500 clips run one persistent launch on 126 CUs with the producers on
    the rest, 1000 and 2100 clips (more recurrence workgroups than the chip has CUs) run as slices.
    No hand-off may time out, and sampled clips equal the same clip alone.  2.5 s clips (T = 125)."""
    m = _model()
    n = 40000
    g = torch.Generator(device="cuda").manual_seed(5)
    for B in (500, 1000, 2100):
        w = (0.1 * torch.randn(B, 2, n, device="cuda", generator=g)).clamp_(-1, 1)
        full = m.probs(w)
        m.synchronize()  # raises if any ready-flag wait timed out
        assert full["probs"].shape == (B, 125, 256)
        _same_as_alone(m, w, full, (0, B // 2, B - 1))
        for k in ("probs", "p_now", "p_future", "vad", "H", "loss"):
            assert torch.isfinite(full[k]).all(), (B, k)
        del w, full
        torch.cuda.empty_cache()


def test_handoff_timeout_is_reported(drop_ready):
    """A ready flag that never arrives (test ABI vap_test_drop_ready) makes the recurrence's bounded
    wait give up after ~2 s: synchronize() raises, and so does the next forward if not checked; the
    word is cleared once reported."""
    m = _model()
    w = _batch(2, 80000, 50)  # 5 s: T = 250, several time chunks
    m(w)
    with pytest.raises(RuntimeError, match="timed out"):
        m.synchronize()
    m.synchronize()  # reported once, then clear
    m(w)
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="timed out"):
        m(w)  # the previous call's failure surfaces here


def test_stream_above_cap_recomputes(monkeypatch):
    """A stream whose recurrence would exceed the cap runs full-recompute pushes (sliced forwards of
    the window, no carry-over) and still equals a full forward of the rolled window."""
    monkeypatch.setenv("VAP_LSTM_MAX_WG", "1")
    m = _model()
    B, window, hop = 12, 48000, 16000  # 24 sequences: 2 workgroups > 1
    st = m.stream(B, context_time=window / 16000, hop_time=hop / 16000)
    assert st.reused_rows == 0
    audio = _batch(B, 2 * hop, 10)
    win = torch.zeros(B, 2, window, device="cuda")
    for k in range(2):
        blk = audio[..., k * hop:(k + 1) * hop]
        out = st.push(blk, full=True)
        win = torch.cat([win[..., hop:], blk], dim=-1)
        ref = m(win)
        assert torch.equal(out["logits"], ref["logits"]), k
    st.synchronize()


def test_heads_per_chunk_equals_once(monkeypatch):
    """By default the fused heads kernel runs per back-end time chunk (frame ranges of every clip);
    VAP_HEADS_CHUNKED=0 runs it once after the last chunk.  The heads are row-wise, so every output
    is bit-identical between the two.  20 s clips: chunks of 640 and 360 frames."""
    w = _batch(3, 320000, 900)
    monkeypatch.setenv("VAP_HEADS_CHUNKED", "0")
    ref = _model().probs(w)
    monkeypatch.setenv("VAP_HEADS_CHUNKED", "1")
    out = _model().probs(w)
    for k in ref:
        assert torch.equal(out[k], ref[k]), k


def test_block_fused_projections_equal_separate(monkeypatch):
    """In the time-chunked back end each layer's block kernel also computes the next layer's
    LayerNorm'd Q/K/V and raw-row cross K/V (k_block.hip, BlockArgs.np); VAP_BLOCK_FUSE=0 runs the
    separate lnproj launches.  Same LayerNorm, same bf16 rounding, same k-step order: bit-identical."""
    w = _batch(3, 320000, 901)
    monkeypatch.setenv("VAP_BLOCK_FUSE", "0")
    ref = _model().probs(w)
    monkeypatch.setenv("VAP_BLOCK_FUSE", "1")
    out = _model().probs(w)
    for k in ref:
        assert torch.equal(out[k], ref[k]), k


def test_bf16_repeat_determinism_and_xcd_handshake():
    """Repeated forwards are bit-identical (the pair recurrence's exchange protocol and the
    hand-counted vmcnt waits leave no race), and the XCD handshake of the last pair launch keeps
    the exchange in L2 exactly when both halves of a pair share an XCD."""
    import ctypes
    from voiceactivityprojection_amd import _native as N

    m = _model()
    for n in (37391, 320000):  # the short golden-clip length (T < 128 schedule) and 20 s (time-chunked)
        w = _batch(2, n, 40)
        ref = m.probs(w)
        for _ in range(3):
            out = m.probs(w)
            for k in ref:
                assert torch.equal(out[k], ref[k]), (n, k)
    m.synchronize()
    buf = np.zeros(64, dtype=np.uint32)
    N.check(N.lib().vap_test_read_lstm_xcc(ctypes.c_void_p(buf.ctypes.data)))
    rec = [int(v) for v in buf if v]
    assert rec, "no handshake record"
    for v in rec:
        own, partner, l2 = v & 255, (v >> 8) & 255, (v >> 16) & 1
        assert l2 == int(own == partner), (own, partner, l2)


def test_exchange_policy_does_not_change_outputs():
    """The pair recurrence's h exchange policy (XCD-local L2 by handshake, forced write-through with
    vap_test_lstm_xplain -1) changes where the bytes travel, not the arithmetic: outputs bit-identical."""
    import ctypes

    from voiceactivityprojection_amd import _native as N

    m = _model()
    w = _batch(3, 160000, 77)
    ref = m.probs(w)
    h = m._native(torch.device("cuda", torch.cuda.current_device()))
    N.check(N.lib().vap_test_lstm_xplain(h, -1))
    out = m.probs(w)
    m.synchronize()
    for k in ref:
        assert torch.equal(out[k], ref[k]), k


def test_exchange_tags_across_launch_sizes_and_wrap():
    """The pair recurrence's exchange slots are never cleared between launches; every launch takes the
    next block of strictly increasing tags, so a slot left by an earlier launch of any length or
    batch can never hold a tag a later launch waits for.  Long large-batch, then small, then short
    large-batch launches give the same outputs as a fresh model; so does a launch that crosses the
    32-bit tag wrap (the engine then clears the slots and restarts the tags)."""
    import ctypes

    from voiceactivityprojection_amd import _native as N

    m, fresh = _model(), _model()
    long = _batch(20, 320000, 300)  # 2000 recurrence steps, 40 sequences
    small = _batch(1, 40960, 320)
    short = _batch(20, 40960, 340)
    m.probs(long)
    for _ in range(5):
        m.probs(small)
    out = m.probs(short)
    m.synchronize()
    ref = fresh.probs(short)
    for k in ref:
        assert torch.equal(out[k], ref[k]), k
    h = m._native(torch.device("cuda", torch.cuda.current_device()))
    N.check(N.lib().vap_test_xtag(h, 0xFFFFFFFF - 1500, None))
    out = m.probs(long)  # needs 2001 tags: wraps
    m.synchronize()
    got = ctypes.c_int64()
    N.check(N.lib().vap_test_xtag(h, -1, ctypes.byref(got)))
    assert 0 < got.value < 10000, got.value
    ref = fresh.probs(long)
    for k in ref:
        assert torch.equal(out[k], ref[k]), k


def test_first_forward_equals_later():
    """The first forward of a fresh model (cold caches, slow DMA) equals the later ones bit for bit.
    It did not: the gate-projection GEMM's second ping-pong wave group waited for its own LDS-DMA of
    stage k+1 one barrier after the first group began reading it, and a late piece was read stale
    (k_gemm2.hip RAW note; 20 clips: 40 sequences, a partial recurrence group)."""
    m = _model()
    w = _batch(20, 320000, 300)
    first = m.probs(w)
    later = m.probs(w)
    m.synchronize()
    for k in first:
        assert torch.equal(first[k], later[k]), k


def test_back_end_split_bit_identical(monkeypatch):
    """The time-chunked back end runs in clip groups on two or three streams (VAP_BE_SPLIT, VAP_BE_FRAC:
    the caller stream's share); every kernel is per sequence and cross attention stays inside a group,
    so the outputs are bit-identical to the one-stream back end whatever the grouping."""
    w = _batch(7, 320000, 505)
    monkeypatch.setenv("VAP_BE_SPLIT", "1")
    ref = _model().probs(w)
    for split, frac in (("2", "0.5"), ("2", "0.3"), ("3", "0.5")):
        monkeypatch.setenv("VAP_BE_SPLIT", split)
        monkeypatch.setenv("VAP_BE_FRAC", frac)
        m = _model()
        out = m.probs(w)
        m.synchronize()
        for k in ref:
            assert torch.equal(out[k], ref[k]), (split, frac, k)


def test_long_clip_schedule_bit_identical(monkeypatch):
    """Clips longer than 1200 frames get their own time chunking (an extra 120-frame first front-end
    piece, back-end chunks shrinking toward the end); the outputs do not depend on the chunking."""
    w = _batch(2, 960000, 77)  # 60 s: T = 3000
    ref = _model().probs(w)  # automatic long-clip chunks
    monkeypatch.setenv("VAP_TC_BE", "0.64")
    monkeypatch.setenv("VAP_TC_FE", "0.1,0.27,0.48,0.72")
    m = _model()
    out = m.probs(w)
    m.synchronize()
    for k in ref:
        assert torch.equal(out[k], ref[k]), k
