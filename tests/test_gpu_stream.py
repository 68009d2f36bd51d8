"""Rolling-window streaming: VapStream against a full forward of the same window.

The reference's streaming loop (sds/run_sds.py:206-241) rolls each new block into a fixed window
and runs model.probs on the whole window.  The engine's stream carries the CPC conv rows that stay
inside the window over between pushes (bf16, hop of whole 160-sample rows) and recomputes the
rest; every conv row is computed by the same kernels with the same per-row arithmetic, so the
stream must be BIT-IDENTICAL to vap_forward on the rolled window, which the parity suite pins to the
reference (tests/test_gpu_parity.py).
"""
import numpy as np
import pytest
import torch

from voiceactivityprojection_amd.weights import synthetic_state_dict, synthetic_waveform

pytestmark = pytest.mark.gpu


def _model(precision):
    from vap.model import VapGPT

    m = VapGPT(precision=precision)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0).items()}, strict=True)
    return m.to("cuda").eval()


@pytest.fixture(scope="module")
def m16():
    return _model("bf16")


@pytest.fixture(scope="module")
def m32():
    return _model("fp32")


def _audio(B, n, seed):
    return torch.from_numpy(np.stack([synthetic_waveform(seed + b, n) for b in range(B)])).cuda()


def _run(model, B, window, hop, pushes, check_at, seed=100):
    st = model.stream(B, context_time=window / 16000, hop_time=hop / 16000)
    audio = _audio(B, hop * pushes, seed)
    win = torch.zeros(B, 2, window, device="cuda")
    for k in range(pushes):
        blk = audio[..., k * hop:(k + 1) * hop]
        out = st.push(blk, full=True)
        win = torch.cat([win[..., hop:], blk], dim=-1)  # x.roll(-hop); x[..., -hop:] = blk
        if k in check_at:
            ref = model(win)
            assert torch.equal(out["logits"], ref["logits"]), f"logits differ at push {k}"
            assert torch.equal(out["vad_logits"], ref["vad"]), f"vad differs at push {k}"
    return st, win


def test_stream_bit_identical_bf16(m16):
    """10 s window, 1 s hop: pushes 0 (full recompute), 1 (first carry-over), 9 (window just full)
    and 11 (every row has been carried over at least once)."""
    st, _ = _run(m16, 3, 160000, 16000, 12, {0, 1, 9, 11})
    assert st.reused_rows > 800, st.reused_rows  # 10 s window: conv4 rows [1, 899) carried over
    g = st.graph_info()  # pushes 1.. ran as captured hipGraphs (one per gate-ring state)
    assert g["replays"] == 11 and g["graphs"] == 10 and g["handoff_error"] == 0, g


def test_stream_graph_replays_bit_identical(m16):
    """Every captured state replayed at least once more (the ring state repeats every 10 pushes):
    replayed graphs stay bit-identical to a full forward of the window."""
    st, _ = _run(m16, 2, 160000, 16000, 24, {12, 21, 23}, seed=300)
    g = st.graph_info()
    assert g["graphs"] == 10 and g["replays"] == 23 and g["handoff_error"] == 0, g


def test_stream_bit_identical_fp32(m32):
    """fp32 parity mode recomputes the window on every push."""
    st, _ = _run(m32, 2, 48000, 16000, 4, {0, 3})
    assert st.reused_rows == 0


def test_stream_odd_hop_bf16(m16):
    """A hop that is not a whole number of 160-sample CPC rows cannot carry rows over: full recompute."""
    st, _ = _run(m16, 2, 64000, 12345, 3, {2})
    assert st.reused_rows == 0


def test_stream_push_semantics(m16):
    """push() returns the window's last hop frames of probs() -- the slice run.py step_extraction
    appends per fold -- and reset() starts again from a zero window."""
    B, W, hop = 2, 160000, 16000
    st = m16.stream(B, context_time=10.0, hop_time=1.0)
    audio = _audio(B, 3 * hop, 7)
    win = torch.zeros(B, 2, W, device="cuda")
    for k in range(3):
        blk = audio[..., k * hop:(k + 1) * hop]
        out = st.push(blk)
        win = torch.cat([win[..., hop:], blk], dim=-1)
    ref = m16.probs(win)
    for key in ("probs", "vad", "p_now", "p_future", "H"):
        assert out[key].shape[1] == 50
        assert torch.equal(out[key], ref[key][:, -50:]), key
    st.reset()
    blk = audio[..., :hop]
    out = st.push(blk, full=True)
    win = torch.cat([torch.zeros(B, 2, W - hop, device="cuda"), blk], dim=-1)
    assert torch.equal(out["logits"], m16(win)["logits"])
    with pytest.raises(ValueError):
        st.push(audio[..., :hop - 1])


def test_stream_bench_shape(m16):
    """C5's per-GPU shape (128 streams x 10 s window, 1 s hop) after the window has filled."""
    st, win = _run(m16, 128, 160000, 16000, 11, {10}, seed=1000)
    assert st.frames == 500
