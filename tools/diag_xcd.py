#!/usr/bin/env python3
"""XCD handshake check (GPU box): the short golden clip through VapGPT.probs N times, VAD error vs
the golden fixture each time, and the pair-LSTM XCC ids of the last launch.

    VAP_LSTM_XPLAIN=0|1|-1 python tools/diag_xcd.py [N]
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from vap.model import VapGPT
    from voiceactivityprojection_amd import _native as N
    from voiceactivityprojection_amd.weights import synthetic_state_dict

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    g = dict(np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "short_clip.npz")))
    m = VapGPT(precision="bf16")
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0).items()}, strict=True)
    m = m.to("cuda").eval()
    w = torch.from_numpy(g["waveform"]).cuda()
    errs = []
    for i in range(n):
        out = m.probs(w)
        m.synchronize()
        errs.append(float(np.abs(out["vad"].float().cpu().numpy() - g["vad"]).max()))
    buf = np.zeros(64, dtype=np.uint32)
    try:
        N.check(N.lib().vap_test_read_lstm_xcc(ctypes.c_void_p(buf.ctypes.data)))
    except (AttributeError, RuntimeError, KeyError):
        pass  # an older library without the record
    rec = [(b, int(v) & 255, (int(v) >> 8) & 255, (int(v) >> 16) & 1) for b, v in enumerate(buf) if v]
    print(f"XPLAIN={os.environ.get('VAP_LSTM_XPLAIN', '0')} vad max err per run: {['%.4f' % e for e in errs]}")
    print("blocks (b, xcc, partner xcc, l2):", rec)


if __name__ == "__main__":
    main()
