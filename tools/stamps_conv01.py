#!/usr/bin/env python3
"""Phase timing of the fused conv0/conv1 kernel (v2) from in-kernel s_memtime stamps (GPU box).

    VAP_CONV01_STAMPS=1 python tools/stamps_conv01.py

Stamps per sampled workgroup: start | prologue done | per phase: SV ready, G ready, k-steps done |
stores issued + drained.  Printed as cycle deltas (shader clock).
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("VAP_CONV01_STAMPS", "1")


def main():
    from vap.model import VapGPT
    from voiceactivityprojection_amd import _native as N
    from voiceactivityprojection_amd.weights import synthetic_batch, synthetic_state_dict

    dev = torch.device("cuda", 0)
    model = VapGPT(precision="bf16")
    model.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0).items()}, strict=True)
    model = model.to(dev).eval()
    wav = torch.from_numpy(synthetic_batch(0, 64, 320000)).to(dev)
    for _ in range(int(os.environ.get("REPS", "3"))):
        model.probs(wav)
    torch.cuda.synchronize()
    buf = np.zeros((8, 24), dtype=np.uint64)
    N.check(N.lib().vap_test_read_stamps(ctypes.c_void_p(buf.ctypes.data)))
    # start | waveform in LDS | split-sample rows | slices 0, 1 | units 0-7, 8-15, 16-23, 24-31 | epilogue
    names, n = ["wv_load", "sv_build", "slices01", "u0_7", "u8_15", "u16_23", "u24_31", "epilogue"], 9
    for i in range(8):
        st = buf[i].astype(np.int64)
        d = np.diff(st[:n])
        ghz = (st[n - 1] - st[0]) / max(1, st[23] - st[22]) * 0.1
        print(f"wg{i}: total {st[n - 1] - st[0]:7d} | " + " ".join(f"{k}={v}" for k, v in zip(names, d)) + f" | clock {ghz:.2f} GHz")


if __name__ == "__main__":
    main()
