"""Rolling-window streaming probabilities.

The reference streams by keeping a fixed-length stereo window, rolling each new audio block into
its end and running ``model.probs`` on the whole window (sds/run_sds.py:206-241
``TurnTakingSDS.add_audio_bytes_to_tensor`` / ``run``); offline, ``run.py:23-131 step_extraction``
keeps the last ``step_time`` frames of each fold.  :class:`VapStream` is that loop on the engine's
``vap_stream_*`` C ABI (include/vap_hip.h): the window lives on the device (zeros at creation, as
``torch.zeros`` in run_sds.py:174), and each :meth:`push` returns the new hop's frames.

In bf16 mode with a hop of whole CPC rows (160 samples) the engine carries the LSTM gate
projections of every conv row whose receptive field stays inside the window over from the
previous push, so only the new audio (plus the zero-padded first row) runs through the CPC conv
stack; the recurrence (zero state at the window start) and the transformer are recomputed, as in
the reference.  The outputs equal a full forward of the same window.
"""
import ctypes
from typing import Dict, Optional

import torch
from torch import Tensor

from . import _native as N


class VapStream:
    """``push(audio[B, 2, hop])`` -> the window's last hop of probs / vad / p_now / p_future / H."""

    def __init__(self, model, batch: int, context_time: float = 10.0, hop_time: float = 1.0,
                 device: Optional[torch.device] = None, now_lims=(0, 1), future_lims=(2, 3)):
        if device is None:
            device = next(iter(model.parameters())).device if any(True for _ in model.parameters()) \
                else torch.device("cuda", torch.cuda.current_device())
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("VapStream needs the MI355X engine (a cuda/HIP device)")
        self.model = model
        self.device = device
        self.batch = int(batch)
        self.window_samples = int(round(context_time * model.sample_rate))
        self.hop_samples = int(round(hop_time * model.sample_rate))
        self.hop_frames = int(round(hop_time * model.frame_hz))
        if self.batch <= 0 or not 0 < self.hop_samples <= self.window_samples:
            raise ValueError(f"bad stream geometry: batch {batch}, window {self.window_samples}, "
                             f"hop {self.hop_samples} samples")
        self.now_lims, self.future_lims = list(now_lims), list(future_lims)
        self._h = model._native(device)
        self._key = model._handle_key
        s = ctypes.c_void_p()
        N.check(N.lib().vap_stream_create(self._h, self.batch, self.window_samples, self.hop_samples,
                                          N.stream_ptr(device), ctypes.byref(s)), "vap_stream_create")
        self._s = s
        frames, reused = ctypes.c_int(), ctypes.c_int64()
        N.check(N.lib().vap_stream_info(self._s, ctypes.byref(frames), None, None, ctypes.byref(reused), None),
                "vap_stream_info")
        self.frames = frames.value
        self.reused_rows = reused.value  # conv4 rows carried over per push (0: full recompute)
        if self.hop_frames > self.frames:
            raise ValueError("hop longer than the window's frames")
        self.pushes = 0
        # persistent outputs: the engine replays a captured hipGraph per state, whose nodes write
        # fixed addresses (vap_stream_graphs)
        self._logits = torch.empty(self.batch, self.frames, 256, device=device)
        self._vad_logits = torch.empty(self.batch, self.frames, 2, device=device)

    def graph_info(self) -> Dict[str, int]:
        """hipGraph replay state: graphs captured, pushes replayed, hand-off error word (synchronous)."""
        g, r, e = ctypes.c_int(), ctypes.c_int64(), ctypes.c_int()
        N.check(N.lib().vap_stream_graphs(self._s, ctypes.byref(g), ctypes.byref(r), ctypes.byref(e)),
                "vap_stream_graphs")
        return {"graphs": g.value, "replays": r.value, "handoff_error": e.value}

    def synchronize(self):
        """Wait for the pushes so far and raise if one of their hand-off waits timed out
        (otherwise reported by the next push)."""
        self._check_handle()
        N.check(N.lib().vap_synchronize(self._h, N.stream_ptr(self.device)), "vap_synchronize")

    def _check_handle(self):
        if self._s is None:
            raise RuntimeError("stream closed")
        if self.model._handle is not self._h or self.model._handle_key != self._key:
            raise RuntimeError("the model's weights or precision changed since the stream was created; "
                               "create a new stream")

    @torch.no_grad()
    def push(self, audio: Tensor, full: bool = False, check: bool = True) -> Dict[str, Tensor]:
        """Roll ``audio`` ([B, 2, hop] float32; channels as in ``VapGPT.forward``) into the window and
        return the last ``hop_frames`` frames of probs (B, F, 256), vad, p_now, p_future (B, F, 2) and
        H (B, F).  ``full=True`` returns every frame of the window plus its ``logits`` / ``vad_logits``.

        ``check=True`` (default) waits for the push and raises if one of its recurrence hand-offs
        timed out, so no invalid hop is ever returned; ``check=False`` returns without waiting (the
        failure then surfaces from the next push or :meth:`synchronize`), for pipelined callers."""
        self._check_handle()
        if audio.dim() != 3 or audio.shape[0] != self.batch or audio.shape[1] != 2 or \
                audio.shape[2] != self.hop_samples:
            raise ValueError(f"expected audio of shape ({self.batch}, 2, {self.hop_samples}), got {tuple(audio.shape)}")
        audio = audio.to(device=self.device, dtype=torch.float32).contiguous()
        B, T = self.batch, self.frames
        dev = self.device
        logits, vad_logits = self._logits, self._vad_logits
        st = N.stream_ptr(dev)
        N.check(N.lib().vap_stream_push(self._s, audio.data_ptr(), logits.data_ptr(), vad_logits.data_ptr(), st),
                "vap_stream_push")
        self.pushes += 1
        probs = torch.empty_like(logits)
        vad = torch.empty(B, T, 2, device=dev)
        p_now = torch.empty(B, T, 2, device=dev)
        p_future = torch.empty(B, T, 2, device=dev)
        H = torch.empty(B, T, device=dev)
        N.check(N.lib().vap_probs(logits.data_ptr(), vad_logits.data_ptr(), B, T, self.model.objective.n_bins,
                                  self.now_lims[0], self.now_lims[-1], self.future_lims[0], self.future_lims[1],
                                  probs.data_ptr(), vad.data_ptr(), p_now.data_ptr(), p_future.data_ptr(),
                                  H.data_ptr(), st), "vap_probs")
        out = {"probs": probs, "vad": vad, "p_now": p_now, "p_future": p_future, "H": H}
        if check:
            N.check(N.lib().vap_synchronize(self._h, st), "vap_synchronize")
        if full:
            out["logits"], out["vad_logits"] = logits.clone(), vad_logits.clone()
            return out
        f = self.hop_frames
        return {k: v[:, -f:] for k, v in out.items()}

    def reset(self):
        """Window back to zeros (a new conversation); the next push recomputes every row."""
        self._check_handle()
        N.check(N.lib().vap_stream_reset(self._s, N.stream_ptr(self.device)), "vap_stream_reset")
        self.pushes = 0

    def close(self):
        if getattr(self, "_s", None) is not None:
            torch.cuda.synchronize(self.device)
            N.lib().vap_stream_destroy(self._s)
            self._s = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
