#!/usr/bin/env python3
"""Standalone resident-LSTM timing (GPU box): S sequences x T steps, nothing else on the GPU.

    python tools/mb_lstm.py [--S 128] [--T 2000]
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from voiceactivityprojection_amd import _native as N
    ap = argparse.ArgumentParser()
    ap.add_argument("--S", type=int, default=128)
    ap.add_argument("--T", type=int, default=2000)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--variant", type=int, default=2, help="0 resident, 2 resident pre-scaled (the engine's)")
    args = ap.parse_args()
    lib = N.lib()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    S, T = args.S, args.T
    gx = (torch.randn(S, T, 1024, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    whh = (torch.randn(1024, 256, generator=g) / 16).to(dev)
    whp = torch.empty(1024 * 256, dtype=torch.bfloat16, device=dev)
    out = torch.empty(S, T, 256, dtype=torch.bfloat16, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    N.check(lib.vap_test_lstm(1, P(gx), S, T, P(whh), P(whp), P(out), args.variant, st))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        N.check(lib.vap_test_lstm(1, P(gx), S, T, P(whh), P(whp), P(out), args.variant, st))
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    print(f"resident LSTM S={S} T={T}: {ms:.3f} ms per launch (incl. W_hh packing), {ms * 1e3 / T:.3f} us per step")
    if os.environ.get("VAP_LSTM_STAMPS"):
        import numpy as np
        buf = np.zeros((8, 4, 5), dtype=np.uint64)
        N.check(lib.vap_test_read_lstm_stamps(ctypes.c_void_p(buf.ctypes.data)))
        b = buf.astype(np.int64)
        print("per step [ksteps+cell, barrier1, h write, barrier2 | step] (shader clocks)")
        for wg in range(min(8, (S + 15) // 16)):
            parts = []
            for k in range(4):
                x = b[wg, k]
                nxt = b[wg, k + 1, 0] - x[0] if k < 3 else 0
                parts.append(f"[{x[1]-x[0]:5d} {x[2]-x[1]:5d} {x[3]-x[2]:5d} {x[4]-x[3]:5d} | {nxt:5d}]")
            print(f"wg{wg}: " + " ".join(parts))


if __name__ == "__main__":
    main()
