#!/usr/bin/env python3
"""Generate golden vectors by running the REFERENCE implementation (build container only).

Imports ``/root/reference`` (read-only) exactly as SURVEY.md §8(c) describes:
  * shim 1 — stub ``torchaudio`` modules in ``sys.modules`` (imported at module import by
    vap/audio.py:2-4; never called on the forward path);
  * shim 2 — replace ``vap.encoder.load_CPC`` (encoder_components.py:179-402, whose fallback
    fetches a checkpoint from the network) with a local constructor of the reference's own
    ``CPCModel(CPCEncoder(256), CPCAR(256, 256, False, n_levels, "LSTM"))``.
Weights are the deterministic synthetic ones from ``voiceactivityprojection_amd.weights`` loaded
with ``strict=True``.  Outputs land in ``tests/golden/*.npz`` (inputs + expected outputs only).

Usage:  python tools/gen_golden.py            (takes ~1 min on 8 CPU threads)
        python tools/gen_golden.py attention  (only the attention-map fixture)
        python tools/gen_golden.py mono       (only the VapGPTMono fixture)
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("VAP_REFERENCE", "/root/reference")
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)

from voiceactivityprojection_amd.weights import synthetic_state_dict, synthetic_waveform  # noqa: E402


def import_reference(lstm_layers: int = 1):
    for name in ["torchaudio", "torchaudio.functional", "torchaudio.transforms"]:
        sys.modules.setdefault(name, types.ModuleType(name))
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import vap.encoder as enc
    from vap.encoder_components import CPCAR, CPCEncoder, CPCModel

    def local_cpc(load_state_dict=True):
        return CPCModel(CPCEncoder(256), CPCAR(256, 256, False, lstm_layers, mode="LSTM"))

    enc.load_CPC = local_cpc
    from vap.model import VapConfig, VapGPT

    return VapGPT, VapConfig


def build_model(lstm_layers: int = 1):
    VapGPT, VapConfig = import_reference(lstm_layers)
    model = VapGPT(VapConfig())
    sd = {k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0, lstm_layers=lstm_layers).items()}
    model.load_state_dict(sd, strict=True)
    return model.eval()


def run(model, wav: np.ndarray, taps: bool = False):
    x = torch.from_numpy(wav)
    store = {}
    hooks = []
    if taps:
        hooks.append(model.encoder.register_forward_hook(
            lambda m, i, o: store.setdefault("enc", []).append(o.detach().clone())))
        hooks.append(model.encoder.encoder.gAR.register_forward_hook(
            lambda m, i, o: store.setdefault("lstm", []).append(o.detach().clone())))
        hooks.append(model.ar_channel.register_forward_hook(
            lambda m, i, o: store.setdefault("ar_channel", []).append(o["x"].detach().clone())))
    with torch.no_grad():
        fw = model(x)
        out = model.probs(x)
    for h in hooks:
        h.remove()
    res = {k: v.numpy() for k, v in out.items()}
    res["logits"] = fw["logits"].numpy()
    res["vad_logits"] = fw["vad"].numpy()
    if taps:
        res["enc1"], res["enc2"] = store["enc"][0].numpy(), store["enc"][1].numpy()
        res["lstm1"] = store["lstm"][0].numpy()
        res["ar_channel1"] = store["ar_channel"][0].numpy()
    return res


def wav_stats(w: np.ndarray):
    return np.array([w.astype(np.float64).sum(), (w.astype(np.float64) ** 2).sum()], dtype=np.float64)


def main():
    torch.set_num_threads(8)
    torch.manual_seed(0)
    os.makedirs(OUT, exist_ok=True)
    model = build_model(1)

    # (a) per-stage taps, one short stereo clip (2.56 s -> T = 128)
    n = 40960
    wav = synthetic_waveform(100, n)[None]
    r = run(model, wav, taps=True)
    np.savez_compressed(
        os.path.join(OUT, "short_clip.npz"), waveform=wav, clip_index=100,
        probs=r["probs"], vad=r["vad"], p_now=r["p_now"], p_future=r["p_future"], H=r["H"], loss=r["loss"],
        logits=r["logits"], vad_logits=r["vad_logits"], enc1=r["enc1"], enc2=r["enc2"],
        lstm1_head=r["lstm1"][:, :64], ar_channel1=r["ar_channel1"])

    # (b) B = 2 x 20 s, inputs regenerated from clip seeds 0, 1 (only checksums stored)
    n = 320000
    wav = np.stack([synthetic_waveform(i, n) for i in (0, 1)])
    r = run(model, wav)
    np.savez_compressed(
        os.path.join(OUT, "batch_20s.npz"), clip_start=0, n_samples=n, wav_stats=wav_stats(wav),
        wav_head=wav[:, :, :16], vad=r["vad"], p_now=r["p_now"], p_future=r["p_future"], H=r["H"],
        loss=r["loss"], probs_head=r["probs"][:, :8], probs_tail=r["probs"][:, -8:],
        logits_tail=r["logits"][:, -4:])

    # (c) long context 60 s (AliBi extrapolation, T = 3000), clip seed 7
    n = 960000
    wav = synthetic_waveform(7, n)[None]
    r = run(model, wav)
    np.savez_compressed(
        os.path.join(OUT, "long_60s.npz"), clip_start=7, n_samples=n, wav_stats=wav_stats(wav),
        vad=r["vad"], p_now=r["p_now"], p_future=r["p_future"], H=r["H"], loss=r["loss"],
        probs_tail=r["probs"][:, -4:])

    # (d) ragged lengths: the example wav length at 16 kHz (37392 -> T 117), T = 1001, minimum T = 101
    for name, n, seed in (("len_37392", 37392, 11), ("len_320319", 320319, 12), ("len_min", 32320, 13)):
        wav = synthetic_waveform(seed, n)[None]
        r = run(model, wav)
        keep = {"waveform": wav} if n < 100000 else {"clip_start": seed, "n_samples": n, "wav_stats": wav_stats(wav)}
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **keep, vad=r["vad"], p_now=r["p_now"],
                            p_future=r["p_future"], H=r["H"], loss=r["loss"], probs_tail=r["probs"][:, -4:])

    # too-short clip: reference raises (quirk Q2) -- record the message
    try:
        run(model, synthetic_waveform(14, 32000)[None])
        short_err = ""
    except RuntimeError as e:  # expected
        short_err = str(e)

    # (e) two-layer LSTM variant (open item O1)
    model2 = build_model(2)
    wav = synthetic_waveform(100, 40960)[None]
    r = run(model2, wav)
    np.savez_compressed(os.path.join(OUT, "lstm2_short.npz"), waveform=wav, probs=r["probs"], vad=r["vad"],
                        p_now=r["p_now"], p_future=r["p_future"], H=r["H"], loss=r["loss"], logits=r["logits"])

    # (f) label-extraction KATs via the reference objective (integer / bit-exact)
    from vap.utils import vad_list_to_onehot

    obj = model.objective
    vas, names = [], []
    ex = json.load(open(os.path.join(REF, "example", "student_long_female_en-US-Wavenet-G_vad_list.json")))
    vas.append(vad_list_to_onehot(ex, duration=2.337, frame_hz=50).numpy()); names.append("example")
    import csv

    with open(os.path.join(REF, "dataset_phrases", "phrases.csv")) as f:
        rows = list(csv.DictReader(f))
    for row in rows[::15]:
        vl = json.loads(row["vad_list"])
        dur = float(row["scp"]) + 2.5
        vas.append(vad_list_to_onehot(vl, duration=dur, frame_hz=50).numpy()); names.append(row["name"])
    rng = np.random.default_rng(5)
    for T in (101, 117, 250, 1000):
        runs = np.cumsum(rng.integers(1, 40, size=(2, T)), axis=1)
        va = np.zeros((T, 2), dtype=np.float32)
        for c in range(2):
            flips = np.zeros(T, dtype=np.int64)
            idx = runs[c][runs[c] < T]
            flips[idx] = 1
            va[:, c] = (np.cumsum(flips) % 2).astype(np.float32)
        vas.append(va); names.append(f"random_binary_{T}")
    kat = {}
    for i, (nm, va) in enumerate(zip(names, vas)):
        lab = obj.get_labels(torch.from_numpy(va)[None]).numpy()
        kat[f"va_{i}"] = va
        kat[f"labels_{i}"] = lab
    # soft (sigmoid-like) VA, as used inside probs() (quirk Q1)
    soft = rng.random((3, 400, 2)).astype(np.float32)
    kat["soft_va"] = soft
    kat["soft_labels"] = obj.get_labels(torch.from_numpy(soft)).numpy()
    kat["names"] = np.array(names)
    np.savez_compressed(os.path.join(OUT, "labels_kat.npz"), **kat)

    meta = {"short_clip_error": short_err, "lstm_layers_default": 1, "seed": 0,
            "generator": "voiceactivityprojection_amd.weights (splitmix64 counter streams)",
            "torch": torch.__version__, "reference": REF}
    with open(os.path.join(OUT, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", sorted(os.listdir(OUT)))


def gen_attention():
    """(g) VapGPT.forward(attention=True) maps (model.py:264-267) of a 0.8 s clip (T = 40): every
    layer's self / cross / cross-self softmax weights, (1, 2, L, H, T, T)."""
    torch.set_num_threads(8)
    model = build_model(1)
    n = 12800
    wav = synthetic_waveform(21, n)[None]
    with torch.no_grad():
        out = model(torch.from_numpy(wav), attention=True)
    np.savez_compressed(os.path.join(OUT, "attention_maps.npz"), waveform=wav, logits=out["logits"].numpy(),
                        vad_logits=out["vad"].numpy(), self_attn=out["self_attn"].numpy(),
                        cross_attn=out["cross_attn"].numpy(), cross_self_attn=out["cross_self_attn"].numpy())
    print("wrote attention_maps.npz", {k: tuple(v.shape) for k, v in out.items()})


def gen_mono():
    """(h) VapGPTMono (vap/model.py:271-393) with va_history (5 bins): forward + probs of a 2.56 s mono
    clip with a seeded binary VA track and its history bins."""
    torch.set_num_threads(8)
    import_reference(1)
    from vap.model import VapGPTMono, VapMonoConfig

    model = VapGPTMono(VapMonoConfig(va_history=True, va_history_bins=5))
    sd = {k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0, mono=True, va_history_bins=5).items()}
    model.load_state_dict(sd, strict=True)
    model.eval()
    n = 40960
    wav = synthetic_waveform(40, n, channels=1)[None]
    T = 128
    rng = np.random.default_rng(41)
    va = (rng.random((1, T, 2)) < 0.4).astype(np.float32)
    hist = rng.random((1, T, 5)).astype(np.float32)
    with torch.no_grad():
        out = model(torch.from_numpy(wav), torch.from_numpy(va), torch.from_numpy(hist))
        pr = model.probs(torch.from_numpy(wav), torch.from_numpy(va))  # probs() passes no history
    np.savez_compressed(os.path.join(OUT, "mono.npz"), waveform=wav, va=va, va_history=hist,
                        logits=out["logits"].numpy(), probs_logits_nohist=pr["probs"].numpy(),
                        p_now=pr["p_now"].numpy(), p_future=pr["p_future"].numpy(), H=pr["H"].numpy())
    print("wrote mono.npz", out["logits"].shape)


def gen_bench4():
    """(i) The bench configuration's clips (BASELINE configs[1]: 20 s stereo, clip seeds 0..3 of the
    bench's own synthetic_batch): every per-frame output in full, the 256-way probs on every 10th
    frame, so the bf16 perf path is pinned to the reference directly (not to the engine's fp32 mode)."""
    torch.set_num_threads(8)
    model = build_model(1)
    from voiceactivityprojection_amd.weights import synthetic_batch

    n = 320000
    wav = synthetic_batch(0, 4, n)
    r = run(model, wav)
    np.savez_compressed(
        os.path.join(OUT, "bench4_20s.npz"), clip_start=0, n_samples=n, wav_stats=wav_stats(wav),
        vad=r["vad"], p_now=r["p_now"], p_future=r["p_future"], H=r["H"], loss=r["loss"],
        probs_stride10=r["probs"][:, ::10], vad_logits=r["vad_logits"])
    print("wrote bench4_20s.npz", r["probs"].shape)


EXAMPLE_WAV = "student_long_female_en-US-Wavenet-G.wav"


def gen_example():
    """(j) BASELINE configs[0] (run.py:190-279 on example/student_long_female_en-US-Wavenet-G.wav): the
    reference VapGPT.probs on the waveform exactly as the build's run.py feeds it (the build's
    load_waveform: int16 / 32768, 24 -> 16 kHz sinc resample; mono -> zero second channel,
    run.py:219-221).  The resampler is the build's restatement of torchaudio's (absent here), so
    RESAMPLING is unpinned; this fixture pins everything after it.  The wav itself is copied next to
    the fixture (tests/golden/, a reference data file) because the GPU box has no /root/reference."""
    import shutil

    torch.set_num_threads(8)
    from voiceactivityprojection_amd.audio import load_waveform

    src = os.path.join(REF, "example", EXAMPLE_WAV)
    shutil.copyfile(src, os.path.join(OUT, EXAMPLE_WAV))
    x, sr = load_waveform(src, sample_rate=16000)
    if x.shape[0] == 1:
        x = torch.cat((x, torch.zeros_like(x)))
    wav = x.unsqueeze(0).numpy()
    model = build_model(1)
    r = run(model, wav)
    np.savez_compressed(os.path.join(OUT, "example_wav.npz"), waveform=wav, sample_rate=sr,
                        probs=r["probs"], vad=r["vad"], p_now=r["p_now"], p_future=r["p_future"], H=r["H"],
                        loss=r["loss"])
    print("wrote example_wav.npz", wav.shape, r["probs"].shape)


def gen_utils():
    """(k) The reference's host VAD utilities (vap/utils.py:21-49, 170-272) on seeded binary VAD: run
    lengths, silence filling / spike omission at several limits, onehot <-> list conversions.  The
    build's voiceactivityprojection_amd/utils.py and the native vad_post_kernel are pinned to them."""
    import_reference(1)
    from vap import utils as U

    rng = np.random.default_rng(9)
    cases = {}
    for i, T in enumerate((1, 7, 60, 333)):
        runs = rng.integers(1, 9, size=(2, T))
        va = np.zeros((T, 2), dtype=np.float32)
        for c in range(2):
            edges = np.cumsum(runs[c])
            flips = np.zeros(T, dtype=np.int64)
            flips[edges[edges < T]] = 1
            va[:, c] = ((np.cumsum(flips) + c) % 2).astype(np.float32)
        cases[f"va_{i}"] = va
        idx, dur, val = U.find_island_idx_len(torch.from_numpy(va[:, 0]))
        cases[f"island_{i}"] = np.stack([idx.numpy(), dur.numpy(), val.numpy().astype(np.int64)])
        for fill, omit in ((0.02, 0.02), (0.06, 0.1), (0.2, 0.04)):
            v = U.vad_fill_silences(torch.from_numpy(va.copy()), max_fill_time=fill, frame_hz=50)
            v = U.vad_omit_spikes(v, max_omit_time=omit, frame_hz=50)
            cases[f"post_{i}_{fill}_{omit}"] = v.numpy()
        lists = U.vad_onehot_to_vad_list(torch.from_numpy(va[None]), frame_hz=50, ipu_thresh_time=0.1)
        cases[f"list_{i}"] = np.array(json.dumps(lists))
        back = U.vad_list_to_onehot(lists[0], duration=T / 50, frame_hz=50)
        cases[f"onehot_{i}"] = back.numpy()
    np.savez_compressed(os.path.join(OUT, "vad_utils.npz"), **cases)
    print("wrote vad_utils.npz", len(cases))


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which == "attention":
        gen_attention()
    elif which == "mono":
        gen_mono()
    elif which == "bench4":
        gen_bench4()
    elif which == "example":
        gen_example()
    elif which == "utils":
        gen_utils()
    else:
        main()
        gen_attention()
        gen_mono()
        gen_bench4()
        gen_example()
        gen_utils()
