#!/usr/bin/env python3
"""Recurrence hand-off timeline of the bench forward (GPU box): when the pair recurrence's workgroup 0
started, waited for each front-end piece (ready) and published each chunk (done), us from its start.

    VAP_LSTM_HANDOFF=1 python tools/handoff.py [--batch 64] [--seconds 20]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("VAP_LSTM_HANDOFF", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    from vap.model import VapGPT
    from voiceactivityprojection_amd import _native as N
    from voiceactivityprojection_amd.weights import synthetic_batch, synthetic_state_dict

    dev = torch.device("cuda", 0)
    model = VapGPT(precision="bf16")
    model.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0).items()}, strict=True)
    model = model.to(dev).eval()
    wav = torch.from_numpy(synthetic_batch(0, args.batch, int(args.seconds * 16000))).to(dev)
    buf = np.zeros(49, dtype=np.uint64)
    # back to back like bench.py: events around each forward, one synchronize at the end
    model.probs(wav)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.iters + 1)]
    ev[0].record()
    for it in range(args.iters):
        model.probs(wav)
        ev[it + 1].record()
    torch.cuda.synchronize()
    times = [ev[i].elapsed_time(ev[i + 1]) for i in range(args.iters)]
    N.check(N.lib().vap_test_read_lstm_handoff(ctypes.c_void_p(buf.ctypes.data)))
    b = buf.astype(np.int64)
    t0 = b[0]
    rows = []
    for c in range(16):
        w, r, d = b[1 + 3 * c], b[2 + 3 * c], b[3 + 3 * c]
        if d <= 0 or d < t0:
            break
        rows.append(f"c{c}: wait {(w - t0) / 100:7.1f} ready {(r - t0) / 100:7.1f} (stall {(r - w) / 100:6.1f}) done {(d - t0) / 100:7.1f}")
    print("last forward:")
    for x in rows:
        print("   ", x)
    print(f"{args.iters} forwards: min {min(times):.3f} median {sorted(times)[len(times) // 2]:.3f} ms")


if __name__ == "__main__":
    main()
