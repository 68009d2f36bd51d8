"""ctypes binding of libvap_hip.so (C ABI: include/vap_hip.h).

There is no CPU fallback: if the library is missing or no HIP device is present, every entry
point raises.  Build the library with ``python -c "import __graft_entry__ as g; g.build()"`` or
``make -C voiceactivityprojection_amd/csrc``.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
# VAP_LIB_AB=<name> loads _lib/<name> instead (A/B timing of two builds of the engine on one box;
# the name must be a file in _lib, so the package never loads a library from elsewhere)
VAP_LIB_AB = os.environ.get("VAP_LIB_AB", "")
LIB_PATH = os.path.join(_HERE, "_lib", os.path.basename(os.environ.get("VAP_LIB_AB", "")) or "libvap_hip.so")

VAP_OK, VAP_ERR_INVALID, VAP_ERR_TOO_SHORT, VAP_ERR_HIP, VAP_ERR_WEIGHTS, VAP_ERR_UNSUPPORTED = range(6)
PRECISION = {"fp32": 0, "bf16": 1}
KERNEL_CLASS = {"conv0": 1, "conv1": 2, "conv234": 3, "lstm_proj": 4, "lstm_rec": 5, "downsample": 6,
                "tr_gemm": 7, "attn": 8, "norm": 9, "heads": 10, "probs": 11}


class VapDims(ctypes.Structure):
    _fields_ = [("dim", ctypes.c_int), ("num_heads", ctypes.c_int), ("channel_layers", ctypes.c_int),
                ("cross_layers", ctypes.c_int), ("lstm_layers", ctypes.c_int), ("n_bins", ctypes.c_int),
                ("precision", ctypes.c_int), ("mono", ctypes.c_int), ("va_history_bins", ctypes.c_int)]


class NativeLibraryMissing(ImportError):
    pass


_lib: Optional[ctypes.CDLL] = None

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_SIGS = {
    "vap_create": (ctypes.c_int, [ctypes.POINTER(VapDims), ctypes.POINTER(_P)]),
    "vap_destroy": (None, [_P]),
    "vap_num_params": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int)]),
    "vap_param_info": (ctypes.c_int, [_P, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(_I64)]),
    "vap_set_param": (ctypes.c_int, [_P, ctypes.c_char_p, _P, _I64, _P]),
    "vap_finalize": (ctypes.c_int, [_P, _P]),
    "vap_frame_lengths": (ctypes.c_int, [_I64, ctypes.POINTER(_I64)]),
    "vap_workspace_size": (ctypes.c_int, [_P, ctypes.c_int, _I64, ctypes.POINTER(ctypes.c_size_t)]),
    "vap_forward": (ctypes.c_int, [_P, _P, ctypes.c_int, _I64, _P, _P, _P, ctypes.c_size_t, _P]),
    "vap_forward_attention": (ctypes.c_int, [_P, _P, ctypes.c_int, _I64, _P, _P, _P, _P, _P, _P, ctypes.c_size_t, _P]),
    "vap_forward_mono": (ctypes.c_int, [_P, _P, _P, _P, ctypes.c_int, _I64, _P, _P, ctypes.c_size_t, _P]),
    "vap_encode_va": (ctypes.c_int, [_P, _P, _P, ctypes.c_int, _P, _P]),
    "vap_encode": (ctypes.c_int, [_P, _P, ctypes.c_int, _I64, _P, _P, ctypes.c_size_t, _P]),
    "vap_stream_create": (ctypes.c_int, [_P, ctypes.c_int, _I64, _I64, _P, _P]),
    "vap_stream_push": (ctypes.c_int, [_P, _P, _P, _P, _P]),
    "vap_stream_info": (ctypes.c_int, [_P, _P, _P, _P, _P, _P]),
    "vap_stream_reset": (ctypes.c_int, [_P, _P]),
    "vap_stream_graphs": (ctypes.c_int, [_P, _P, _P, _P]),
    "vap_stream_destroy": (None, [_P]),
    "vap_probs": (ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, _P, _P, _P, _P, _P, _P]),
    "vap_aggregate": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, _P]),
    "vap_probs_loss": (ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int, _P, ctypes.c_float, _P, _P, _P, _P, _P, _P, _P, _P]),
    "vap_labels_loss": (ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.c_int, _P, ctypes.c_int, ctypes.c_float, _P, _P,
                                       _P]),
    "vap_vad_postprocess": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int,
                                           ctypes.c_int, _P, _P]),
    "vap_synchronize": (ctypes.c_int, [_P, _P]),
    "vap_test_plan": (ctypes.c_int, [_P, ctypes.c_int, _I64, _P]),
    "vap_test_xtag": (ctypes.c_int, [_P, _I64, ctypes.POINTER(_I64)]),
    "vap_test_drop_ready": (ctypes.c_int, [_P, ctypes.c_int]),
    "vap_test_lstm_xplain": (ctypes.c_int, [_P, ctypes.c_int]),
    "vap_timing": (ctypes.c_int, [_P, ctypes.c_int]),
    "vap_timing_read": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]),
    "vap_test_gemm": (ctypes.c_int, [ctypes.c_int, _P, _I64, _I64, _P, ctypes.c_int, ctypes.c_int, _P, ctypes.c_int,
                                     ctypes.c_int, _P, _I64, _I64, _P, _I64, _I64, _P, _P, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, _P]),
    "vap_test_attention": (ctypes.c_int, [ctypes.c_int, _P, _I64, _I64, _P, _I64, _I64, _P, _I64, _I64, _P, _I64,
                                          _I64, _P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_float, _P]),
    "vap_test_lstm": (ctypes.c_int, [ctypes.c_int, _P, ctypes.c_int, ctypes.c_int, _P, _P, _P, ctypes.c_int, _P]),
    "vap_test_conv0": (ctypes.c_int, [ctypes.c_int, _P, ctypes.c_int, _I64, ctypes.c_int, _P, _P, _P, _P, _P, _P]),
    "vap_test_layernorm": (ctypes.c_int, [ctypes.c_int, _P, _I64, _P, _P, _P, _P, _P]),
    "vap_test_read_stamps": (ctypes.c_int, [_P]),
    "vap_test_read_block_stamps": (ctypes.c_int, [_P]),
    "vap_test_read_lnproj_stamps": (ctypes.c_int, [_P]),
    "vap_test_read_gemm_stamps": (ctypes.c_int, [_P]),
    "vap_test_read_lstm_stamps": (ctypes.c_int, [_P]),
    "vap_test_heads": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "vap_test_read_lstm_handoff": (ctypes.c_int, [_P]),
    "vap_test_read_lstm_xcc": (ctypes.c_int, [_P]),
    "vap_test_pack_weight": (ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.c_int, _P]),
    "vap_test_block": (ctypes.c_int, [_P, _P, ctypes.c_int, _P, _P, _P, _P, _P, ctypes.c_int, _P]),
    "vap_test_lnproj": (ctypes.c_int, [_P, _P, ctypes.c_int, _P, _P, ctypes.c_int, _P, ctypes.c_int, _P, _P, _P, _P, _P]),
    "vap_test_lnproj_packed": (ctypes.c_int, [_P, _P, ctypes.c_int, _P, _P, ctypes.c_int, _P, ctypes.c_int, _P, _P, _P, _P, _P]),
    "vap_test_block_packed": (ctypes.c_int, [_P, _P, ctypes.c_int, _P, _P, _P, _P, _P, ctypes.c_int, _P]),
    "vap_test_probe_mfma_f32": (ctypes.c_int, [_P, _P, _P, _P]),
    "vap_test_convk4": (ctypes.c_int, [_P, _I64, ctypes.c_int, _P, _P, _P, _P, _P, _I64, ctypes.c_int, ctypes.c_int, _P]),
    "vap_test_convk4_stamps": (ctypes.c_int, [_P]),
    "vap_last_error": (ctypes.c_char_p, []),
    "vap_build_info": (ctypes.c_char_p, []),
}
EXPORTED = sorted(_SIGS)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryMissing(
                f"libvap_hip.so not found at {LIB_PATH}: the MI355X engine has no CPU fallback. "
                "Build it with `make -C voiceactivityprojection_amd/csrc` (hipcc, gfx950).")
        l = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(l, name, None)
            if fn is None:
                if VAP_LIB_AB:  # an older build under A/B may lack newer test entry points
                    continue
                raise NativeLibraryMissing(
                    f"{LIB_PATH} does not export {name} (declared in include/vap_hip.h): the library is stale; "
                    "rebuild it with `make -C voiceactivityprojection_amd/csrc`.")
            fn.restype = res
            fn.argtypes = args
        _lib = l
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc == VAP_OK:
        return
    msg = lib().vap_last_error().decode(errors="replace")
    if what:
        msg = f"{what}: {msg}"
    if rc == VAP_ERR_TOO_SHORT:
        raise RuntimeError(msg)
    if rc == VAP_ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    if rc == VAP_ERR_INVALID:
        raise ValueError(msg)
    raise RuntimeError(msg)


def frame_lengths(n_samples: int):
    arr = (_I64 * 6)()
    check(lib().vap_frame_lengths(int(n_samples), arr), "vap_frame_lengths")
    return [int(v) for v in arr]


def ptr(t) -> int:
    return t.data_ptr()


def stream_ptr(device=None) -> int:
    import torch

    return torch.cuda.current_stream(device).cuda_stream
