"""Host-side helpers mirroring reference vap/utils.py (JSON I/O, determinism switch, VAD lists).

These are plumbing around the hot path (run.py's I/O contract); the VAD
post-processing used by ``VapGPT.vad`` runs natively (vap_vad_postprocess), the tensor versions
here keep the reference's utility API for callers that use them directly.
"""
from __future__ import annotations

import json
from typing import List, Tuple

import torch
from torch import Tensor

VAD_LIST = List[List[List[float]]]


def frame_lengths(n_samples: int) -> List[int]:
    """Output lengths of conv0..conv4 and the 50 Hz frame count T for ``n_samples`` per channel
    (host arithmetic, no device): the CPC conv specs (k, s, p) = (10, 5, 3), (8, 4, 2), (4, 2, 1) x 3
    (vap/encoder_components.py:83-92) and the causal downsample k5 s2, left pad 4
    (vap/encoder.py:24-31, CConv1d vap/encoder_components.py:454-460).  Same chain as the engine's
    vap_frame_lengths."""
    lens = []
    n = int(n_samples)
    for k, st, pd in ((10, 5, 3), (8, 4, 2), (4, 2, 1), (4, 2, 1), (4, 2, 1)):
        n = (n + 2 * pd - k) // st + 1 if n + 2 * pd >= k else 0
        lens.append(n)
    lens.append((n + 4 - 5) // 2 + 1 if n > 0 else 0)
    return lens


def time_to_frames(t: float, hop_time: float) -> int:
    """vap/audio.py:19-20."""
    return int(t / hop_time)


def add_zero_channel(w: Tensor) -> Tensor:
    """utils.py:15-18."""
    return torch.cat((w, torch.zeros_like(w)), dim=-2)


def find_island_idx_len(x: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    """Run-length encoding of a 1-D tensor, as the reference's helper returns it (vap/utils.py:21-49):
    (start index of every run, its length, its value)."""
    assert x.ndim == 1
    values, lengths = torch.unique_consecutive(x, return_counts=True)
    starts = torch.cumsum(lengths, 0) - lengths
    return starts, lengths, values


def everything_deterministic():
    """The reference switches torch to deterministic algorithms at import (vap/utils.py:52-103).  The
    engine's kernels are deterministic by construction (fixed reduction order, no float atomics);
    this applies the same switch to any torch code around them."""
    import os

    os.environ["CUBLAS_WORKSPACE_CONFIG"] = ":4096:8"
    torch.backends.cudnn.deterministic = True
    torch.use_deterministic_algorithms(mode=True)


def batch_to_device(batch, device="cuda"):
    return {k: (v.to(device) if isinstance(v, Tensor) else v) for k, v in batch.items()}


def _jsonable(v):
    if isinstance(v, Tensor):
        return v.tolist()
    if isinstance(v, dict):
        return {k: _jsonable(x) for k, x in v.items()}
    return v


def tensor_dict_to_json(d):
    """Tensors (also inside nested dicts) -> nested lists, for run.py's JSON (vap/utils.py:116-124)."""
    return _jsonable(d)


def vad_list_to_onehot(vad_list: VAD_LIST, duration: float, hop_time: float = 0, frame_hz: float = 0,
                       channel_first: bool = False) -> Tensor:
    """VAD segment list [[(start, end), ...] per speaker] -> (n_frames, 2) 0/1 frames, a frame being
    active when it lies in [frame(start), frame(end)) with frame(t) = int(t / hop) (vap/utils.py:170-195)."""
    assert hop_time > 0 or frame_hz > 0, "vad_list_to_onehot requires `frame_hz` or `hop_time`"
    hop = 1 / frame_hz if frame_hz > 0 else hop_time
    frames = torch.arange(time_to_frames(duration, hop))
    cols = []
    for ch in range(2):
        on = torch.zeros(frames.shape[0], dtype=torch.bool)
        for seg in (vad_list[ch] if ch < len(vad_list) else []):
            on |= (frames >= time_to_frames(seg[0], hop)) & (frames < time_to_frames(seg[1], hop))
        cols.append(on)
    out = torch.stack(cols, dim=-1).to(torch.float32)
    return out.t() if channel_first else out


def vad_onehot_to_vad_list(vad: Tensor, frame_hz: int = 50, ipu_thresh_time: float = 0.1) -> List[VAD_LIST]:
    """(B, n_frames, 2) 0/1 frames -> per clip and speaker a list of [start, end] seconds (2 decimals);
    a segment starting less than ``ipu_thresh_time`` after the previous segment's end is merged into
    it (vap/utils.py:198-236)."""
    assert vad.ndim == 3, f"Expects vad with batch-dim of shape (B, n_frames, 2) but got {vad.shape}"
    result = []
    for clip in vad:
        speakers = []
        for ch in range(2):
            starts, lengths, values = find_island_idx_len(clip[:, ch])
            on = values == 1
            t0 = (starts[on] / frame_hz).tolist()
            t1 = (starts[on] / frame_hz + lengths[on] / frame_hz).tolist()
            segs, prev_end = [], None
            for a, b in zip(t0, t1):
                a, b = round(a, 2), round(b, 2)
                if prev_end is not None and a - prev_end < ipu_thresh_time:
                    segs[-1][1] = b
                else:
                    segs.append([a, b])
                prev_end = b
            speakers.append(segs)
        result.append(speakers)
    return result


def _replace_short_runs(vad: Tensor, max_frames: int, run_value: float, new_value: float) -> Tensor:
    """In place, per speaker column: every run of ``run_value`` at most ``max_frames`` long becomes
    ``new_value``."""
    for ch in range(vad.shape[-1]):
        _, lengths, values = find_island_idx_len(vad[:, ch])
        short = (values == run_value) & (lengths <= max_frames)
        vad[torch.repeat_interleave(short, lengths), ch] = new_value
    return vad


def vad_fill_silences(vad: Tensor, max_fill_time: float = 0.02, frame_hz: float = 50) -> Tensor:
    """Silences of at most ``max_fill_time`` become speech (vap/utils.py:239-255)."""
    assert vad.ndim == 2 and vad.shape[-1] == 2, f"Expects (N_FRAMES, 2) got {vad.shape}"
    return _replace_short_runs(vad, round(max_fill_time * frame_hz), 0.0, 1.0)


def vad_omit_spikes(vad: Tensor, max_omit_time: float = 0.02, frame_hz: float = 50) -> Tensor:
    """Speech spikes of at most ``max_omit_time`` become silence (vap/utils.py:258-272)."""
    assert vad.ndim == 2 and vad.shape[-1] == 2, f"Expects (N_FRAMES, 2) got {vad.shape}"
    return _replace_short_runs(vad, round(max_omit_time * frame_hz), 1.0, 0.0)


def write_json(data, filename):
    with open(filename, "w", encoding="utf-8") as jsonfile:
        json.dump(data, jsonfile, ensure_ascii=False)


def read_json(path, encoding="utf8"):
    with open(path, "r", encoding=encoding) as f:
        return json.loads(f.read())
