#!/usr/bin/env python3
"""Per-step phase timing of the resident bf16 LSTM (steps 100..103) from s_memtime stamps (GPU box).

    VAP_LSTM_STAMPS=1 python tools/stamps_lstm.py
Runs a few stream pushes (128 streams, 10 s window: the transformer runs beside the recurrence)
and then one small forward (B = 4: the recurrence mostly alone), printing the stamps after each.
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("VAP_LSTM_STAMPS", "1")


def show(N, tag):
    buf = np.zeros((8, 4, 5), dtype=np.uint64)
    N.check(N.lib().vap_test_read_lstm_stamps(ctypes.c_void_p(buf.ctypes.data)))
    b = buf.astype(np.int64)
    print(f"== {tag}: per step [ksteps+cell, barrier1, h write, barrier2 | step]")
    for wg in range(8):
        if b[wg, 0, 0] == 0:
            continue
        parts = []
        for k in range(4):
            s = b[wg, k]
            nxt = b[wg, k + 1, 0] if k < 3 else 0
            parts.append(f"[{s[1]-s[0]:5d} {s[2]-s[1]:5d} {s[3]-s[2]:5d} {s[4]-s[3]:5d} | {nxt - s[0] if k < 3 else 0:5d}]")
        print(f"wg{wg}: " + " ".join(parts))
    buf[:] = 0


def main():
    from vap.model import VapGPT
    from voiceactivityprojection_amd import _native as N
    from voiceactivityprojection_amd.weights import synthetic_state_dict, synthetic_waveform

    dev = torch.device("cuda", 0)
    m = VapGPT(precision="bf16")
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0).items()}, strict=True)
    m = m.to(dev).eval()
    B, hop = 128, 16000
    st = m.stream(B, context_time=10.0, hop_time=1.0)
    audio = torch.from_numpy(np.stack([synthetic_waveform(b, 3 * hop) for b in range(B)])).to(dev)
    for k in range(3):
        st.push(audio[..., k * hop:(k + 1) * hop])
    torch.cuda.synchronize()
    show(N, "stream push (128 x 10 s)")
    w = torch.from_numpy(np.stack([synthetic_waveform(b, 160000) for b in range(4)])).to(dev)
    m.probs(w)
    torch.cuda.synchronize()
    show(N, "forward B=4 x 10 s")
    from voiceactivityprojection_amd.weights import synthetic_batch
    wb = torch.from_numpy(synthetic_batch(0, 64, 320000)).to(dev)  # the bench workload
    for _ in range(2):
        m.probs(wb)
    torch.cuda.synchronize()
    show(N, f"bench forward B=64 x 20 s (steps from {os.environ.get('VAP_LSTM_STAMP_T0', '100')})")


if __name__ == "__main__":
    main()
