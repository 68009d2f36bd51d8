"""Audio loading (mirror of reference vap/audio.py:39-69) without torchaudio.

``load_waveform`` reads PCM WAV (scipy.io.wavfile; int16 / int32 / float) into float32 in [-1, 1)
(int16 / 32768 as torchaudio.load's default normalisation) and resamples with a restatement of
torchaudio.functional.resample's default windowed-sinc method (sinc_interp_hann,
lowpass_filter_width=6, rolloff=0.99).  torchaudio is absent in this image, so resample parity is
UNPINNED: no golden vector from the reference covers it.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F


def _sinc_kernel(orig: int, new: int, width_param: int = 6, rolloff: float = 0.99):
    base = min(orig, new) * rolloff
    width = math.ceil(width_param * orig / base)
    idx = torch.arange(-width, width + orig, dtype=torch.float64)[None, None] / orig
    t = torch.arange(0, -new, -1, dtype=torch.float64)[:, None, None] / new + idx
    t = (t * base).clamp_(-width_param, width_param)
    window = torch.cos(t * math.pi / width_param / 2) ** 2
    t = t * math.pi
    kernels = torch.where(t == 0, torch.tensor(1.0, dtype=torch.float64), t.sin() / t)
    kernels = kernels * window * (base / orig)
    return kernels, width


def resample(x: torch.Tensor, orig_freq: int, new_freq: int) -> torch.Tensor:
    if orig_freq == new_freq:
        return x
    g = math.gcd(int(orig_freq), int(new_freq))
    orig, new = int(orig_freq) // g, int(new_freq) // g
    kernel, width = _sinc_kernel(orig, new)
    shape = x.shape
    w = x.reshape(-1, shape[-1]).to(torch.float64)
    n = w.shape[-1]
    w = F.pad(w, (width, width + orig))
    y = F.conv1d(w[:, None], kernel, stride=orig).transpose(1, 2).reshape(w.shape[0], -1)
    y = y[..., : int(math.ceil(new * n / orig))]
    return y.reshape(shape[:-1] + y.shape[-1:]).to(x.dtype)


def load_waveform(path: str, sample_rate: Optional[int] = 16000, start_time: Optional[float] = None,
                  end_time: Optional[float] = None, mono: bool = False) -> Tuple[torch.Tensor, int]:
    from scipy.io import wavfile

    sr, data = wavfile.read(path)
    if data.dtype == np.int16:
        x = data.astype(np.float32) / 32768.0
    elif data.dtype == np.int32:
        x = data.astype(np.float32) / 2147483648.0
    elif data.dtype == np.uint8:
        x = (data.astype(np.float32) - 128.0) / 128.0
    else:
        x = data.astype(np.float32)
    x = torch.from_numpy(x.reshape(len(x), -1).T.copy())  # (channels, samples)
    if start_time is not None or end_time is not None:
        s = int(start_time * sr) if start_time is not None else 0
        e = int(end_time * sr) if end_time is not None else x.shape[-1]
        x = x[:, s:e]
    if mono and x.shape[0] > 1:
        x = x.mean(dim=0).unsqueeze(0)
    if sample_rate is not None and sr != sample_rate:
        x = resample(x, sr, sample_rate)
        sr = sample_rate
    return x, sr
