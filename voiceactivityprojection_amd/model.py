"""Drop-in mirror of the reference model API (vap/model.py) on the MI355X engine.

    from vap.model import VapGPT, VapConfig, VAPModel, load_older_state_dict, BIN_TIMES

* ``VapConfig``      == vap/model.py:42-79 (same fields, same ``--vap_*`` argparse flags).
* ``VapGPT``         == vap/model.py:125-268: same module tree / state-dict keys (``load_state_dict``
  with ``strict=True`` as run.py:199-201), same ``forward`` / ``probs`` / ``vad`` / ``encode_audio``
  signatures, outputs and errors.  Parameters live in ordinary torch Parameters (storage only);
  all compute runs in ``libvap_hip.so`` through the C ABI (include/vap_hip.h).  CPU tensors raise:
  there is no CPU fallback.
* ``VAPModel``       the reference's Lightning training class name (vap/train.py:244), exported
  here as an inference-only alias of VapGPT.

Extra (engine) knobs: ``precision`` ("fp32" parity mode, default; "bf16" perf mode) as a
constructor argument / ``VAP_PRECISION`` env var, and ``lstm_layers`` (inferred from state dicts).
"""


import ctypes
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn
from torch import Tensor

from . import _native as N
from .objective import ObjectiveVAP
from .weights import schema as _schema
from .weights import synthetic_state_dict

BIN_TIMES: list = [0.2, 0.4, 0.6, 0.8]


def load_older_state_dict(path="example/VAP_3mmz3t0u_50Hz_ad20s_134-epoch9-val_2.56.ckpt"):
    """vap/model.py:28-39 (old Lightning checkpoint key remap); safe loader only."""
    sd = torch.load(path, map_location="cpu", weights_only=True)["state_dict"]
    new_sd = {}
    for k, v in sd.items():
        if "VAP.codebook" in k:
            continue
        if "vap_head" in k:
            k = k.replace("vap_head.projection_head", "vap_head")
        new_sd[k.replace("net.", "")] = v
    return new_sd


_SYNC_CHECK = os.environ.get("VAP_SYNC_CHECK", "0") not in ("", "0")


@dataclass
class VapConfig:
    sample_rate: int = 16_000
    frame_hz: int = 50
    bin_times: List[float] = field(default_factory=lambda: BIN_TIMES)

    # Encoder (training flag)
    freeze_encoder: int = 1
    load_pretrained: int = 1

    # GPT
    dim: int = 256
    channel_layers: int = 1
    cross_layers: int = 3
    num_heads: int = 4
    dropout: float = 0.1

    @staticmethod
    def add_argparse_args(parser, fields_added=[]):
        for k, v in VapConfig.__dataclass_fields__.items():
            if k == "bin_times":
                parser.add_argument(f"--vap_{k}", nargs="+", type=float, default=v.default_factory())
            else:
                parser.add_argument(f"--vap_{k}", type=v.type, default=v.default)
            fields_added.append(k)
        return parser, fields_added

    @staticmethod
    def args_to_conf(args):
        return VapConfig(**{k.replace("vap_", ""): v for k, v in vars(args).items() if k.startswith("vap_")})


def _container(root: nn.Module, dotted: str) -> nn.Module:
    mod = root
    for part in dotted.split("."):
        if part not in mod._modules:
            mod.add_module(part, nn.Module())
        mod = mod._modules[part]
    return mod


class VapGPT(nn.Module):
    """vap/model.py:125-268 on the MI355X engine."""

    def __init__(self, conf: Optional[VapConfig] = None, precision: Optional[str] = None, lstm_layers: int = 1):
        super().__init__()
        if conf is None:
            conf = VapConfig()
        self.conf = conf
        self.sample_rate = conf.sample_rate
        self.frame_hz = conf.frame_hz
        self.precision = precision or os.environ.get("VAP_PRECISION", "fp32")
        if self.precision not in N.PRECISION:
            raise ValueError(f"precision must be one of {list(N.PRECISION)}")
        self.lstm_layers = lstm_layers
        self.objective = ObjectiveVAP(bin_times=conf.bin_times, frame_hz=conf.frame_hz)
        self._build_params(lstm_layers)
        self._handle = None
        self._handle_key = None
        self._dirty = True
        self._ws: Optional[Tensor] = None

    # ------------------------------------------------------------------ parameters / state dict
    def _schema_kw(self) -> dict:
        return {}

    def _schema(self, lstm_layers: int):
        c = self.conf
        return _schema(dim=c.dim, channel_layers=c.channel_layers, cross_layers=c.cross_layers,
                       num_heads=c.num_heads, lstm_layers=lstm_layers, n_bins=len(c.bin_times), **self._schema_kw())

    def _build_params(self, lstm_layers: int):
        c = self.conf
        init = synthetic_state_dict(seed=0, dim=c.dim, channel_layers=c.channel_layers,
                                    cross_layers=c.cross_layers, num_heads=c.num_heads,
                                    lstm_layers=lstm_layers, n_bins=len(c.bin_times), **self._schema_kw())
        for key, shape in self._schema(lstm_layers):
            if key == "objective.codebook.emb.weight":
                continue  # owned by ObjectiveVAP.codebook.emb
            prefix, name = key.rsplit(".", 1)
            mod = _container(self, prefix)
            mod.register_parameter(name, nn.Parameter(torch.from_numpy(init[key]).reshape(shape),
                                                      requires_grad=False))
        self.lstm_layers = lstm_layers

    def _drop_lstm(self):
        base = self.encoder.encoder.gAR.baseNet
        for name in list(base._parameters):
            del base._parameters[name]

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        """nn.Module.load_state_dict with the LSTM depth inferred from the keys."""
        n = 0
        while f"encoder.encoder.gAR.baseNet.weight_ih_l{n}" in state_dict:
            n += 1
        if n and n != self.lstm_layers:
            dev = next(self.parameters()).device
            self._drop_lstm()
            self.lstm_layers = n
            p = "encoder.encoder.gAR.baseNet"
            base = self.encoder.encoder.gAR.baseNet
            for key, shape in self._schema(n):
                if key.startswith(p + "."):
                    base.register_parameter(key[len(p) + 1:], nn.Parameter(torch.zeros(shape, device=dev),
                                                                          requires_grad=False))
        res = super().load_state_dict(state_dict, strict=strict, assign=assign)
        self._dirty = True
        return res

    def _apply(self, fn, *args, **kwargs):
        self._dirty = True
        self._ws = None
        return super()._apply(fn, *args, **kwargs)

    def invalidate(self):
        """Call after modifying parameters in place (re-packs the kernel layouts on next use)."""
        self._dirty = True

    def set_precision(self, precision: str):
        if precision not in N.PRECISION:
            raise ValueError(f"precision must be one of {list(N.PRECISION)}")
        self.precision = precision
        self._dirty = True
        self._ws = None

    # ------------------------------------------------------------------ native handle
    def _free_handle(self):
        if self._handle is not None:
            try:
                N.lib().vap_destroy(self._handle)
            except Exception:
                pass
            self._handle = None

    def __del__(self):
        try:
            self._free_handle()
        except Exception:
            pass

    def _native(self, device: torch.device):
        key = (device, self.precision, self.lstm_layers)
        if self._handle is not None and not self._dirty and self._handle_key == key:
            return self._handle
        lib = N.lib()
        self._free_handle()
        c = self.conf
        kw = self._schema_kw()
        dims = N.VapDims(c.dim, c.num_heads, c.channel_layers, c.cross_layers, self.lstm_layers,
                         len(c.bin_times), N.PRECISION[self.precision], int(kw.get("mono", False)),
                         int(kw.get("va_history_bins", 0)))
        h = ctypes.c_void_p()
        N.check(lib.vap_create(ctypes.byref(dims), ctypes.byref(h)), "vap_create")
        self._handle = h
        sd = self.state_dict()
        st = N.stream_ptr(device)
        keep = []
        n = ctypes.c_int()
        N.check(lib.vap_num_params(h, ctypes.byref(n)))
        for i in range(n.value):
            k = ctypes.c_char_p()
            numel = ctypes.c_int64()
            N.check(lib.vap_param_info(h, i, ctypes.byref(k), ctypes.byref(numel)))
            name = k.value.decode()
            if name not in sd:
                raise RuntimeError(f"Missing key in state_dict: {name}")
            t = sd[name]
            if t.device != device:
                raise RuntimeError(f"Expected all tensors to be on the same device, but found {t.device} "
                                   f"(parameter {name}) and {device} (input); call model.to({str(device)!r})")
            t = t.detach().float().contiguous()
            keep.append(t)
            N.check(lib.vap_set_param(h, name.encode(), t.data_ptr(), t.numel(), st), "vap_set_param")
        N.check(lib.vap_finalize(h, st), "vap_finalize")
        del keep
        self._handle_key = key
        self._dirty = False
        return h

    def _workspace(self, h, B: int, n: int, device) -> Tensor:
        need = ctypes.c_size_t()
        N.check(N.lib().vap_workspace_size(h, B, n, ctypes.byref(need)), "vap_workspace_size")
        if self._ws is None or self._ws.numel() < need.value or self._ws.device != device:
            self._ws = None
            self._ws = torch.empty(need.value, dtype=torch.uint8, device=device)
        return self._ws

    def _check_input(self, waveform: Tensor) -> Tensor:
        assert waveform.shape[1] == 2, f"audio VAP ENCODER: {waveform.shape} != (B, 2, n_samples)"
        if not waveform.is_cuda:
            raise RuntimeError("VapGPT (MI355X engine) runs on HIP devices only: move the model and the waveform "
                               "to 'cuda' (there is no CPU fallback)")
        return waveform.float().contiguous()

    # ------------------------------------------------------------------ reference API
    @property
    def horizon_time(self):
        return self.objective.horizon_time

    def encode_audio(self, audio: Tensor) -> Tuple[Tensor, Tensor]:
        """vap/model.py:169-175: EncoderCPC on each speaker -> (x1, x2), each (B, T, 256)."""
        audio = self._check_input(audio)
        B, _, n = audio.shape
        T = N.frame_lengths(n)[-1]
        h = self._native(audio.device)
        ws = self._workspace(h, B, n, audio.device)
        out = torch.empty(2, B, T, self.conf.dim, device=audio.device, dtype=torch.float32)
        N.check(N.lib().vap_encode(h, audio.data_ptr(), B, n, out.data_ptr(), ws.data_ptr(), ws.numel(),
                                   N.stream_ptr(audio.device)), "vap_encode")
        return out[0], out[1]

    def forward(self, waveform: Tensor, attention: bool = False) -> Dict[str, Tensor]:
        """vap/model.py:249-268 -> {"logits": (B, T, 256), "vad": (B, T, 2)}; with ``attention=True`` also
        "self_attn" (B, 2, channel_layers, H, T, T), "cross_attn" and "cross_self_attn"
        (B, 2, cross_layers, H, T, T): the softmax weights of every layer (model.py:264-267)."""
        if attention:
            return self._forward_attention(waveform)
        waveform = self._check_input(waveform)
        B, _, n = waveform.shape
        T = N.frame_lengths(n)[-1]
        if T <= 0:
            raise RuntimeError(f"waveform of {n} samples is too short for one frame")
        h = self._native(waveform.device)
        ws = self._workspace(h, B, n, waveform.device)
        logits = torch.empty(B, T, self.objective.n_classes, device=waveform.device, dtype=torch.float32)
        vad = torch.empty(B, T, 2, device=waveform.device, dtype=torch.float32)
        N.check(N.lib().vap_forward(h, waveform.data_ptr(), B, n, logits.data_ptr(), vad.data_ptr(), ws.data_ptr(),
                                    ws.numel(), N.stream_ptr(waveform.device)), "vap_forward")
        if _SYNC_CHECK:
            self.synchronize(waveform.device)
        return {"logits": logits, "vad": vad}

    def synchronize(self, device=None) -> None:
        """Wait for the engine's work on the current stream and raise if a hand-off of the persistent
        LSTM recurrence timed out since the last check (its outputs would be invalid).  Without this
        call such a failure raises from the next forward on the model.  ``VAP_SYNC_CHECK=1`` runs it
        after every forward (debugging: it costs a device sync per call)."""
        if self._handle is None:
            return
        dev = device if device is not None else self._handle_key[0]
        N.check(N.lib().vap_synchronize(self._handle, N.stream_ptr(dev)), "vap_synchronize")

    def _forward_attention(self, waveform: Tensor) -> Dict[str, Tensor]:
        waveform = self._check_input(waveform)
        B, _, n = waveform.shape
        T = N.frame_lengths(n)[-1]
        if T <= 0:
            raise RuntimeError(f"waveform of {n} samples is too short for one frame")
        c = self.conf
        dev = waveform.device
        h = self._native(dev)
        ws = self._workspace(h, B, n, dev)
        logits = torch.empty(B, T, self.objective.n_classes, device=dev, dtype=torch.float32)
        vad = torch.empty(B, T, 2, device=dev, dtype=torch.float32)
        sa = torch.empty(B, 2, c.channel_layers, c.num_heads, T, T, device=dev, dtype=torch.float32)
        ca = torch.empty(B, 2, c.cross_layers, c.num_heads, T, T, device=dev, dtype=torch.float32)
        csa = torch.empty_like(ca)
        N.check(N.lib().vap_forward_attention(h, waveform.data_ptr(), B, n, logits.data_ptr(), vad.data_ptr(),
                                              sa.data_ptr() if sa.numel() else None,
                                              ca.data_ptr() if ca.numel() else None,
                                              csa.data_ptr() if csa.numel() else None, ws.data_ptr(), ws.numel(),
                                              N.stream_ptr(dev)), "vap_forward_attention")
        return {"logits": logits, "vad": vad, "self_attn": sa, "cross_attn": ca, "cross_self_attn": csa}

    @torch.no_grad()
    def probs(self, waveform: Tensor, vad: Optional[Tensor] = None, now_lims: List[int] = [0, 1],
              future_lims: List[int] = [2, 3], *, out: Optional[Dict[str, Tensor]] = None) -> Dict[str, Tensor]:
        """vap/model.py:180-225, including quirk Q1: labels always come from the model's own sigmoid
        VAD (the ``vad`` argument is shadowed), so ``loss`` is always returned.

        ``out`` (engine extension, keyword only): preallocated contiguous fp32 device tensors for any of
        the six outputs (e.g. views into one packed buffer that a single collective then ships,
        ``distributed.PackedOutputs``); the missing ones are allocated.  The results are returned in
        the same tensors."""
        fw = self(waveform)
        logits, vad_logits = fw["logits"], fw["vad"]
        B, T, C = logits.shape
        dev = logits.device
        obj = self.objective
        if T - 1 < obj.horizon:  # quirk Q2: the reference fails in unfold
            raise RuntimeError(f"maximum size for tensor at dimension 1 is {T - 1} but size is {obj.horizon}")
        n = T - obj.horizon
        shapes = {"probs": (B, T, C), "vad": (B, T, 2), "p_now": (B, T, 2), "p_future": (B, T, 2), "H": (B, T),
                  "loss": (B, n)}
        res = {}
        for k, shape in shapes.items():
            t = out.get(k) if out is not None else None
            if t is None:
                t = torch.empty(shape, device=dev, dtype=torch.float32)
            elif tuple(t.shape) != shape or t.dtype != torch.float32 or t.device != dev or not t.is_contiguous():
                raise ValueError(f"out[{k!r}] must be a contiguous float32 {shape} tensor on {dev}, "
                                 f"got {tuple(t.shape)} {t.dtype} on {t.device}")
            res[k] = t
        labels = torch.empty(B, n, dtype=torch.int64, device=dev)
        st = N.stream_ptr(dev)
        bf = (ctypes.c_int * obj.n_bins)(*obj.bin_frames)
        # softmax / sigmoid / H / p_now / p_future, then labels from the model's own sigmoid VAD (quirk Q1)
        # and loss_vap (objective.py:209-243) in one call
        N.check(N.lib().vap_probs_loss(logits.data_ptr(), vad_logits.data_ptr(), B, T, obj.n_bins, now_lims[0],
                                       now_lims[-1], future_lims[0], future_lims[1], bf, obj.threshold_ratio,
                                       res["probs"].data_ptr(), res["vad"].data_ptr(), res["p_now"].data_ptr(),
                                       res["p_future"].data_ptr(), res["H"].data_ptr(), labels.data_ptr(),
                                       res["loss"].data_ptr(), st), "vap_probs_loss")
        return res

    @torch.no_grad()
    def vad(self, waveform: Tensor, max_fill_silence_time: float = 0.02, max_omit_spike_time: float = 0.02,
            vad_cutoff: float = 0.5) -> Tensor:
        """vap/model.py:227-247: binary VAD with short silences filled and short spikes removed."""
        vl = self(waveform)["vad"]
        B, T, _ = vl.shape
        out = torch.empty_like(vl)
        N.check(N.lib().vap_vad_postprocess(vl.data_ptr(), B, T, float(vad_cutoff),
                                            round(max_fill_silence_time * self.frame_hz),
                                            round(max_omit_spike_time * self.frame_hz), out.data_ptr(),
                                            N.stream_ptr(vl.device)), "vap_vad_postprocess")
        return out


def _stream(self, batch: int, context_time: float = 10.0, hop_time: float = 1.0, **kw):
    """Rolling-window streaming (sds/run_sds.py:206-241; SURVEY config C5): see
    :class:`voiceactivityprojection_amd.stream.VapStream`."""
    from .stream import VapStream

    return VapStream(self, batch, context_time=context_time, hop_time=hop_time, **kw)


VapGPT.stream = _stream


@dataclass
class VapMonoConfig:
    """vap/model.py:82-124 (same fields and defaults)."""
    sample_rate: int = 16_000
    frame_hz: int = 50
    bin_times: List[float] = field(default_factory=lambda: BIN_TIMES)
    mono: bool = True
    va_history: bool = False
    va_history_bins: int = 5

    freeze_encoder: bool = True
    load_pretrained: bool = True

    dim: int = 256
    channel_layers: int = 1
    cross_layers: int = 3
    num_heads: int = 4
    dropout: float = 0.1

    # the reference's argparse helpers iterate and build VapConfig (model.py:101-124); kept as is
    add_argparse_args = staticmethod(VapConfig.add_argparse_args)
    args_to_conf = staticmethod(VapConfig.args_to_conf)


class VapGPTMono(VapGPT):
    """vap/model.py:271-393 on the MI355X engine: one speaker's CPC encoder + VA conditioning
    (``va_condition`` Linear(2, dim) -> ``va_cond_ln``, plus ``va_cond_history`` when
    ``conf.va_history``), ``ar_channel`` and ``ar`` plain GPT stacks, ``vap_head``.  Same state-dict
    keys; forward / probs / encode_audio / encode_va with the reference's signatures."""

    def __init__(self, conf: Optional[VapMonoConfig] = None, precision: Optional[str] = None, lstm_layers: int = 1):
        super().__init__(conf if conf is not None else VapMonoConfig(), precision, lstm_layers)

    def _schema_kw(self) -> dict:
        c = self.conf
        return {"mono": True, "va_history_bins": int(c.va_history_bins) if c.va_history else 0}

    def encode_audio(self, audio: Tensor) -> Tensor:
        """model.py:359-363: (B, 1, N) -> (B, T, 256)."""
        assert audio.shape[1] == 1, f"audio VAP ENCODER: {audio.shape} != (B, 1, n_samples)"
        if not audio.is_cuda:
            raise RuntimeError("VapGPTMono (MI355X engine) runs on HIP devices only (there is no CPU fallback)")
        audio = audio.float().contiguous()
        B, _, n = audio.shape
        T = N.frame_lengths(n)[-1]
        h = self._native(audio.device)
        ws = self._workspace(h, B, n, audio.device)
        out = torch.empty(B, T, self.conf.dim, device=audio.device, dtype=torch.float32)
        N.check(N.lib().vap_encode(h, audio.data_ptr(), B, n, out.data_ptr(), ws.data_ptr(), ws.numel(),
                                   N.stream_ptr(audio.device)), "vap_encode")
        return out

    def encode_va(self, va: Tensor, va_history: Optional[Tensor] = None) -> Tensor:
        """model.py:352-357: LN(va_condition(va) [+ va_cond_history(va_history)])."""
        if not va.is_cuda:
            raise RuntimeError("VapGPTMono (MI355X engine) runs on HIP devices only (there is no CPU fallback)")
        va = va.float().contiguous()
        hist = self._history(va_history, va)
        rows = va.numel() // 2
        out = torch.empty(*va.shape[:-1], self.conf.dim, device=va.device, dtype=torch.float32)
        h = self._native(va.device)
        N.check(N.lib().vap_encode_va(h, va.data_ptr(), hist.data_ptr() if hist is not None else None, rows,
                                      out.data_ptr(), N.stream_ptr(va.device)), "vap_encode_va")
        return out

    def _history(self, va_history: Optional[Tensor], va: Tensor) -> Optional[Tensor]:
        if not (self.conf.va_history and va_history is not None):
            return None  # model.py:355: only with conf.va_history and a history given
        hist = va_history.to(device=va.device, dtype=torch.float32).contiguous()
        if hist.shape[:-1] != va.shape[:-1] or hist.shape[-1] != self.conf.va_history_bins:
            raise RuntimeError(f"va_history {tuple(hist.shape)} does not match va {tuple(va.shape)} "
                               f"x {self.conf.va_history_bins} bins")
        return hist

    def forward(self, waveform: Tensor, va: Tensor, va_history: Optional[Tensor] = None,
                attention: bool = False) -> Dict[str, Tensor]:
        """model.py:365-393 -> {"logits": (B, T, 256), "vad": va}."""
        assert not attention, "Attention Mono model is not implemented"
        assert waveform.shape[1] == 1, f"audio VAP ENCODER: {waveform.shape} != (B, 1, n_samples)"
        if not waveform.is_cuda:
            raise RuntimeError("VapGPTMono (MI355X engine) runs on HIP devices only: move the model and the "
                               "waveform to 'cuda' (there is no CPU fallback)")
        waveform = waveform.float().contiguous()
        B, _, n = waveform.shape
        T = N.frame_lengths(n)[-1]
        if T <= 0:
            raise RuntimeError(f"waveform of {n} samples is too short for one frame")
        if tuple(va.shape) != (B, T, 2):
            raise RuntimeError(f"va {tuple(va.shape)} must be (B, T, 2) = ({B}, {T}, 2) for this waveform")
        dev = waveform.device
        vad = va.to(device=dev, dtype=torch.float32).contiguous()
        hist = self._history(va_history, vad)
        h = self._native(dev)
        ws = self._workspace(h, B, n, dev)
        logits = torch.empty(B, T, self.objective.n_classes, device=dev, dtype=torch.float32)
        N.check(N.lib().vap_forward_mono(h, waveform.data_ptr(), vad.data_ptr(),
                                         hist.data_ptr() if hist is not None else None, B, n, logits.data_ptr(),
                                         ws.data_ptr(), ws.numel(), N.stream_ptr(dev)), "vap_forward_mono")
        return {"logits": logits, "vad": va}

    @torch.no_grad()
    def probs(self, waveform: Tensor, vad: Tensor, now_lims: List[int] = [0, 1],
              future_lims: List[int] = [2, 3]) -> Dict[str, Tensor]:
        """model.py:325-350: probs, vad (the argument), p_now, p_future, H -- no labels / loss."""
        out = self(waveform, vad)
        logits = out["logits"]
        B, T, C = logits.shape
        dev = logits.device
        probs = torch.empty_like(logits)
        p_now = torch.empty(B, T, 2, device=dev)
        p_future = torch.empty(B, T, 2, device=dev)
        H = torch.empty(B, T, device=dev)
        sig = torch.empty(B, T, 2, device=dev)  # vap_probs' sigmoid(vad) slot; the mono model returns vad itself
        zeros = torch.zeros(B, T, 2, device=dev)
        N.check(N.lib().vap_probs(logits.data_ptr(), zeros.data_ptr(), B, T, self.objective.n_bins,
                                  now_lims[0], now_lims[-1], future_lims[0], future_lims[1], probs.data_ptr(),
                                  sig.data_ptr(), p_now.data_ptr(), p_future.data_ptr(), H.data_ptr(),
                                  N.stream_ptr(dev)), "vap_probs")
        return {"probs": probs, "vad": vad, "p_now": p_now, "p_future": p_future, "H": H}

    def vad(self, *args, **kwargs):
        raise AttributeError("VapGPTMono has no VAD head (vap/model.py:271-393)")

    def stream(self, *args, **kwargs):
        raise NotImplementedError("streaming is a VapGPT (stereo) path")


class VAPModel(VapGPT):
    """Inference alias for the reference's ``vap.train.VAPModel`` (vap/train.py:244): a VapGPT."""

    def __init__(self, conf: Optional[VapConfig] = None, *args, **kwargs):
        super().__init__(conf, *args, **kwargs)
