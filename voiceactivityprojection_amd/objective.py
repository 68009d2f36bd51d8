"""VAP objective (mirror of reference vap/objective.py:10-282) over the native kernels.

``get_labels`` and ``probs_next_speaker_aggregate`` run on the MI355X (libvap_hip); they take device
tensors and raise on CPU tensors -- there is no CPU fallback.  ``Codebook.encode/decode`` and
``ProjectionWindow`` are small device-agnostic tensor helpers kept for API parity.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch import Tensor

from . import _native as N
from .weights import bin_frames as _bin_frames
from .weights import code_vectors


def bin_times_to_frames(bin_times: List[float], frame_hz: int) -> List[int]:
    """objective.py:10-11 (float32 product truncated)."""
    return _bin_frames(bin_times, frame_hz)


def _require_device(t: Tensor, what: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(f"{what}: the MI355X VAP engine runs on HIP devices only (got a {t.device} tensor); "
                           "move the tensor to 'cuda'")


class ProjectionWindow:
    """The projection window of objective.py:14-76 as a tensor helper (API parity; the labels of the
    hot path come from the native ``vap_labels_loss``).  For frame t the window is va[t+1 : t+1+horizon]
    split into the bins of ``bin_frames``; a bin is active when its mean activity reaches
    ``threshold_ratio``.  Output (..., n_frames - horizon, 2, n_bins) as float 0/1."""

    def __init__(self, bin_times: List = [0.2, 0.4, 0.6, 0.8], frame_hz: int = 50, threshold_ratio: float = 0.5):
        self.bin_times = bin_times
        self.frame_hz = frame_hz
        self.threshold_ratio = threshold_ratio
        self.bin_frames = bin_times_to_frames(bin_times, frame_hz)
        self.n_bins = len(self.bin_frames)
        self.total_bins = 2 * self.n_bins
        self.horizon = sum(self.bin_frames)

    def projection(self, va: Tensor) -> Tensor:
        """(..., T, 2) -> (..., T - horizon, 2, horizon): the future frames seen from every frame."""
        future = va[..., 1:, :]
        return future.unfold(-2, self.horizon, 1)

    def projection_bins(self, projection_window: Tensor) -> Tensor:
        sums = torch.stack([part.sum(dim=-1) for part in projection_window.split(self.bin_frames, dim=-1)], dim=-1)
        lengths = torch.tensor(self.bin_frames, dtype=sums.dtype, device=sums.device)
        return (sums / lengths >= self.threshold_ratio).to(torch.float32)

    def __call__(self, va: Tensor) -> Tensor:
        return self.projection_bins(self.projection(va))


class Codebook(nn.Module):
    """objective.py:79-146: 2^(2*n_bins) binary code vectors (bit k of the index, LSB first)."""

    def __init__(self, bin_frames):
        super().__init__()
        self.bin_frames = bin_frames
        self.n_bins = len(self.bin_frames)
        self.total_bins = self.n_bins * 2
        self.n_classes = 2 ** self.total_bins
        self.emb = nn.Embedding(num_embeddings=self.n_classes, embedding_dim=self.total_bins)
        self.emb.weight.data = torch.from_numpy(code_vectors(self.total_bins))
        self.emb.weight.requires_grad_(False)

    def encode(self, x: Tensor) -> Tensor:
        """(..., 2, n_bins) binary -> index; equal to the reference's distance argmax for binary x."""
        assert x.shape[-2:] == (2, self.n_bins), f"Codebook expects (..., 2, {self.n_bins}) got {x.shape}"
        w = (2 ** torch.arange(self.total_bins, device=x.device)).view(2, self.n_bins)
        return (x.round().long() * w).sum(dim=(-1, -2))

    def decode(self, idx: Tensor):
        v = self.emb(idx)
        return v.view(*v.shape[:-1], 2, self.n_bins)

    def forward(self, projection_windows: Tensor):
        return self.encode(projection_windows)


class ObjectiveVAP(nn.Module):
    """objective.py:149-282 (metrics helper ``extract_prediction_and_targets`` is out of scope)."""

    def __init__(self, bin_times: List[float] = [0.2, 0.4, 0.6, 0.8], frame_hz: int = 50,
                 threshold_ratio: float = 0.5):
        super().__init__()
        self.frame_hz = frame_hz
        self.bin_times = bin_times
        self.threshold_ratio = threshold_ratio
        self.bin_frames: List[int] = bin_times_to_frames(bin_times, frame_hz)
        self.horizon = sum(self.bin_frames)
        self.horizon_time = sum(bin_times)
        self.codebook = Codebook(self.bin_frames)
        self.projection_window_extractor = ProjectionWindow(bin_times, frame_hz, threshold_ratio)
        self.requires_grad_(False)

    @property
    def n_classes(self) -> int:
        return self.codebook.n_classes

    @property
    def n_bins(self) -> int:
        return self.codebook.n_bins

    def probs_next_speaker_aggregate(self, probs: Tensor, from_bin: int = 0, to_bin: int = 3,
                                     scale_with_bins: bool = False) -> Tensor:
        assert probs.ndim == 3, f"Expected probs of shape (B, n_frames, n_classes) but got {probs.shape}"
        if scale_with_bins:
            raise NotImplementedError("scale_with_bins=True is not on the inference path")
        _require_device(probs, "probs_next_speaker_aggregate")
        p = probs.float().contiguous()
        B, T, _ = p.shape
        out = torch.empty(B, T, 2, device=p.device, dtype=torch.float32)
        N.check(N.lib().vap_aggregate(p.data_ptr(), B, T, self.n_bins, from_bin, to_bin, out.data_ptr(),
                                      N.stream_ptr(p.device)), "vap_aggregate")
        return out

    def window_to_win_dialog_states(self, wins):
        return (wins.sum(-1) > 0).sum(-1)

    def labels_and_loss(self, va: Tensor, logits=None) -> Tuple[Tensor, Tensor]:
        _require_device(va, "get_labels")
        va = va.float().contiguous()
        B, T, _ = va.shape
        n = T - self.horizon
        if T - 1 < self.horizon:
            raise RuntimeError(f"maximum size for tensor at dimension 1 is {T - 1} but size is {self.horizon}")
        labels = torch.empty(B, n, dtype=torch.int64, device=va.device)
        loss = torch.empty(B, n, dtype=torch.float32, device=va.device) if logits is not None else None
        bf = (ctypes.c_int * self.n_bins)(*self.bin_frames)
        N.check(N.lib().vap_labels_loss(logits.data_ptr() if logits is not None else None, va.data_ptr(), B, T, bf,
                                        self.n_bins, self.threshold_ratio, labels.data_ptr(),
                                        loss.data_ptr() if loss is not None else None, N.stream_ptr(va.device)),
                "vap_labels_loss")
        return labels, loss

    def get_labels(self, va: Tensor) -> Tensor:
        """objective.py:209-212: projection-window bits -> codebook index (bit-exact for binary va)."""
        return self.labels_and_loss(va)[0]

    def get_da_labels(self, va: Tensor) -> Tuple[Tensor, Tensor]:
        idx = self.get_labels(va)
        pw = self.projection_window_extractor(va).type(va.dtype)
        return idx, self.window_to_win_dialog_states(pw)

    def loss_vap(self, logits: Tensor, labels: Tensor, reduction: str = "mean") -> Tensor:
        """objective.py:220-243."""
        assert logits.ndim == 3, f"Exptected logits of shape (B, N_FRAMES, N_CLASSES) but got {logits.shape}"
        assert labels.ndim == 2, f"Exptected labels of shape (B, N_FRAMES) but got {labels.shape}"
        nmax = labels.shape[1]
        if logits.shape[1] > nmax:
            logits = logits[:, :nmax]
        loss = F.cross_entropy(logits.reshape(-1, logits.shape[-1]), labels.reshape(-1), reduction=reduction)
        if reduction == "none":
            loss = loss.view(-1, nmax)
        return loss

    def loss_vad(self, vad_output, vad):
        n = vad_output.shape[-2]
        return F.binary_cross_entropy_with_logits(vad_output, vad[:, :n])

    def get_probs(self, logits: Tensor) -> Dict[str, Tensor]:
        assert logits.shape[-1] == self.n_classes
        probs = logits.softmax(dim=-1)
        return {"probs": probs,
                "p_now": self.probs_next_speaker_aggregate(probs, 0, 1),
                "p_future": self.probs_next_speaker_aggregate(probs, 2, 3),
                "p_tot": self.probs_next_speaker_aggregate(probs, 0, 3)}
