#!/usr/bin/env python3
"""Streaming throughput (SURVEY config C5): B streams, each a rolling 10 s window advanced by a 1 s
hop; one push = one step.  Metric: NEW audio-seconds per second (B x hop per step), as C5 counts it.

    python tools/bench_stream.py [--streams 128] [--steps 10] [--warmup 11]

VAP_STREAM_REUSE=0 disables the CPC conv-row carry-over (full recompute per push) for an A/B;
VAP_STREAM_GRAPH=0 issues every push eagerly instead of replaying its captured hipGraph.
Inputs: the seeded synthetic waveform generator (no dataset), bf16, weights random-init.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from vap.model import VapGPT
    from voiceactivityprojection_amd.weights import synthetic_state_dict, synthetic_waveform

    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=128)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=11, help="pushes before timing (10 fill the window)")
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--check-each", action="store_true",
                    help="push(check=True): wait for every push and check its hand-off (the real-time loop's "
                         "default); otherwise pushes are pipelined and checked once after the timed loop")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    m = VapGPT(precision=args.precision)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0).items()}, strict=True)
    m = m.to(dev).eval()
    B, hop = args.streams, 16000
    st = m.stream(B, context_time=10.0, hop_time=1.0)
    n = hop * (args.warmup + args.steps)
    audio = torch.from_numpy(np.stack([synthetic_waveform(5000 + b, n) for b in range(B)])).to(dev)
    for k in range(args.warmup):
        st.push(audio[..., k * hop:(k + 1) * hop], check=args.check_each)
    st.synchronize()
    t0 = time.perf_counter()
    c0 = time.process_time()
    for k in range(args.warmup, args.warmup + args.steps):
        out = st.push(audio[..., k * hop:(k + 1) * hop], check=args.check_each)
    c1 = time.process_time()
    st.synchronize()  # raises if any timed push's hand-off timed out
    dt = (time.perf_counter() - t0) / args.steps
    host_ms = (c1 - c0) / args.steps * 1e3
    print(json.dumps({"metric": "new audio-seconds/sec (streaming, 1 s hop / 10 s window)",
                      "value": round(B * 1.0 / dt, 1), "unit": "audio-s/s", "ms_per_step": round(dt * 1e3, 3),
                      "streams": B, "steps": args.steps, "reused_rows": st.reused_rows, "frames": st.frames,
                      "dtype": args.precision, "data": "synthetic", "checked_each_push": args.check_each,
                      "window_audio_s_per_s": round(B * 10.0 / dt, 1),
                      "host_cpu_ms_per_push": round(host_ms, 3), "graph": st.graph_info()}))


if __name__ == "__main__":
    main()
