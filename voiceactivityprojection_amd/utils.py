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
    """utils.py:21-49: run-length islands (start index, duration, value)."""
    assert x.ndim == 1
    n = len(x)
    y = x[1:] != x[:-1]
    i = torch.cat((torch.where(y)[0], torch.tensor(n - 1, device=x.device).unsqueeze(0))).long()
    it = torch.cat((torch.tensor(-1, device=x.device).unsqueeze(0), i))
    dur = it[1:] - it[:-1]
    idx = torch.cumsum(torch.cat((torch.tensor([0], device=x.device, dtype=torch.long), dur)), dim=0)[:-1]
    return idx, dur, x[i]


def everything_deterministic():
    """utils.py:52-103. The HIP kernels are deterministic by construction (no float atomics, fixed
    reduction order); this keeps the reference's global switch for torch code around them."""
    from os import environ

    environ["CUBLAS_WORKSPACE_CONFIG"] = ":4096:8"
    torch.backends.cudnn.deterministic = True
    torch.use_deterministic_algorithms(mode=True)


def batch_to_device(batch, device="cuda"):
    return {k: (v.to(device) if isinstance(v, Tensor) else v) for k, v in batch.items()}


def tensor_dict_to_json(d):
    new_d = {}
    for k, v in d.items():
        if isinstance(v, Tensor):
            v = v.tolist()
        elif isinstance(v, dict):
            v = tensor_dict_to_json(v)
        new_d[k] = v
    return new_d


def vad_list_to_onehot(vad_list: VAD_LIST, duration: float, hop_time: float = 0, frame_hz: float = 0,
                       channel_first: bool = False) -> Tensor:
    """utils.py:170-195."""
    assert hop_time > 0 or frame_hz > 0, "vad_list_to_onehot requires `frame_hz` or `hop_time`"
    if frame_hz > 0:
        hop_time = 1 / frame_hz
    n_frames = time_to_frames(duration, hop_time)
    vad_tensor = torch.zeros((n_frames, 2))
    for ch, ch_vad in enumerate(vad_list):
        for v in ch_vad:
            s = time_to_frames(v[0], hop_time)
            e = time_to_frames(v[1], hop_time)
            vad_tensor[s:e, ch] = 1.0
    if channel_first:
        vad_tensor = vad_tensor.permute(1, 0)
    return vad_tensor


def vad_onehot_to_vad_list(vad: Tensor, frame_hz: int = 50, ipu_thresh_time: float = 0.1) -> List[VAD_LIST]:
    """utils.py:198-236."""
    assert vad.ndim == 3, f"Expects vad with batch-dim of shape (B, n_frames, 2) but got {vad.shape}"
    batch_vad_list = []
    for b in range(vad.shape[0]):
        vad_list = []
        for ch in range(2):
            idx, dur, val = find_island_idx_len(vad[b, :, ch])
            active = idx[val == 1]
            start_times = active / frame_hz
            ch_vad_list = []
            if len(start_times) == 0:
                vad_list.append(ch_vad_list)
                continue
            end_times = start_times + dur[val == 1] / frame_hz
            start_times, end_times = start_times.tolist(), end_times.tolist()
            s, last_end = round(start_times[0], 2), round(end_times[0], 2)
            ch_vad_list.append([s, last_end])
            for s, e in zip(start_times[1:], end_times[1:]):
                s, e = round(s, 2), round(e, 2)
                if s - last_end < ipu_thresh_time:
                    ch_vad_list[-1][-1] = e
                else:
                    ch_vad_list.append([s, e])
                last_end = e
            vad_list.append(ch_vad_list)
        batch_vad_list.append(vad_list)
    return batch_vad_list


def _fill(vad: Tensor, max_frames: int, value: float) -> Tensor:
    for ch in range(2):
        starts, dur, on_off = find_island_idx_len(vad[:, ch])
        s_ = starts[on_off == (1.0 - value)]
        d_ = dur[on_off == (1.0 - value)]
        w = torch.where(d_ <= max_frames)[0]
        for s, d in zip(s_[w], d_[w]):
            vad[s: s + d, ch] = value
    return vad


def vad_fill_silences(vad: Tensor, max_fill_time: float = 0.02, frame_hz: float = 50) -> Tensor:
    """utils.py:239-255."""
    assert vad.ndim == 2 and vad.shape[-1] == 2, f"Expects (N_FRAMES, 2) got {vad.shape}"
    return _fill(vad, round(max_fill_time * frame_hz), 1.0)


def vad_omit_spikes(vad: Tensor, max_omit_time: float = 0.02, frame_hz: float = 50) -> Tensor:
    """utils.py:258-272."""
    assert vad.ndim == 2 and vad.shape[-1] == 2, f"Expects (N_FRAMES, 2) got {vad.shape}"
    return _fill(vad, round(max_omit_time * frame_hz), 0.0)


def write_json(data, filename):
    with open(filename, "w", encoding="utf-8") as jsonfile:
        json.dump(data, jsonfile, ensure_ascii=False)


def read_json(path, encoding="utf8"):
    with open(path, "r", encoding=encoding) as f:
        return json.loads(f.read())
