"""BASELINE configs end to end on the GPU: C1 (run.py on the reference's example wav) against the
reference's outputs, and the drivers (run.py, bench.py, streaming) refusing to report results of a
forward whose recurrence hand-off timed out."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from voiceactivityprojection_amd.weights import synthetic_waveform

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXAMPLE = os.path.join(REPO, "tests", "golden", "student_long_female_en-US-Wavenet-G.wav")
KEYS = ("probs", "vad", "p_now", "p_future", "H", "loss")


@pytest.mark.parametrize("precision,tol", [("fp32", {"probs": 1e-4, "vad": 1e-4, "p_now": 1e-4, "p_future": 1e-4,
                                                      "H": 1e-3, "loss": 1e-3}),
                                           ("bf16", None)])
def test_run_py_example_wav(tmp_path, golden, precision, tol):
    """BASELINE configs[0] (run.py:190-279): `run.py -a example/student_long_female_en-US-Wavenet-G.wav
    -sd synthetic` writes the JSON the reference writes (keys, nested-list shapes) with values equal to
    the reference's VapGPT.probs on the same 16 kHz waveform (tests/golden/example_wav.npz; the
    24 -> 16 kHz resampler itself is unpinned, torchaudio being absent)."""
    import run
    from test_gpu_parity import BF16_TOL

    tol = tol or BF16_TOL
    g = golden("example_wav")
    out_json = str(tmp_path / "example.json")
    out = run.main(["-a", EXAMPLE, "-sd", "synthetic", "-f", out_json, "--precision", precision])
    data = json.load(open(out_json))
    assert sorted(data) == sorted(KEYS)
    errs = {}
    for k in KEYS:
        got = np.asarray(data[k], dtype=np.float32)
        assert got.shape == g[k].shape, (k, got.shape, g[k].shape)
        np.testing.assert_array_equal(got, out[k].numpy())  # the JSON holds exactly the returned tensors
        errs[k] = float(np.abs(got - g[k]).max())
    bad = {k: e for k, e in errs.items() if not e <= tol[k]}
    assert not bad, f"{precision}: {bad} (all {errs})"
    print(f"run.py example wav {precision} max abs err:", errs)


def test_run_py_raises_on_dropped_handoff(tmp_path, drop_ready):
    """A recurrence hand-off that times out (test ABI vap_test_drop_ready) makes run.main raise
    instead of writing a JSON of invalid outputs."""
    import run
    from scipy.io import wavfile

    wav = synthetic_waveform(60, 80000)  # 5 s stereo: several time chunks
    path = str(tmp_path / "five_s.wav")
    wavfile.write(path, 16000, (wav.T * 32767).astype(np.int16))
    out_json = str(tmp_path / "five_s.json")
    with pytest.raises(RuntimeError, match="timed out"):
        run.main(["-a", path, "-sd", "synthetic", "-f", out_json, "--precision", "bf16"])
    assert not os.path.exists(out_json)


def test_bench_raises_on_dropped_handoff():
    """bench.py fails (non-zero exit, the hand-off error on stderr) rather than printing a number."""
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--batch", "2", "--seconds", "5",
                        "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--no-extras",
                        "--test-drop-ready", "1"], cwd=REPO,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode != 0 and "timed out" in p.stderr, (p.returncode, p.stdout[-500:], p.stderr[-2000:])
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]


def test_stream_push_raises_on_dropped_handoff(drop_ready):
    """VapStream.push checks its hand-off by default (the real-time loop never gets an invalid hop)."""
    from vap.model import VapGPT
    from voiceactivityprojection_amd.weights import synthetic_state_dict

    m = VapGPT(precision="bf16")
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0).items()}, strict=True)
    m = m.to("cuda").eval()
    st = m.stream(2, context_time=5.0, hop_time=1.0)
    blk = torch.from_numpy(np.stack([synthetic_waveform(80 + i, 16000) for i in range(2)])).cuda()
    with pytest.raises(RuntimeError, match="timed out"):
        st.push(blk)
    st.close()


def test_probs_sharded_world1_matches_probs():
    """distributed.probs_sharded on the real engine (world 1, gloo group): the packed single-gather
    path returns exactly model.probs' outputs."""
    import socket

    import torch.distributed as dist
    from vap.model import VapGPT
    from voiceactivityprojection_amd.distributed import probs_sharded
    from voiceactivityprojection_amd.weights import synthetic_state_dict

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        m = VapGPT(precision="bf16")
        m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0).items()}, strict=True)
        m = m.to("cuda").eval()
        w = torch.from_numpy(np.stack([synthetic_waveform(90 + i, 48000) for i in range(3)])).cuda()
        ref = m.probs(w)
        got = probs_sharded(m, w, 0, 1, torch.device("cuda"))
        for k in KEYS:
            assert torch.equal(got[k], ref[k]), k
    finally:
        dist.destroy_process_group()
