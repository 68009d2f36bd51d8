#!/usr/bin/env python3
"""Phase timing of the fused FFN kernel from in-kernel s_memtime stamps (GPU box).

    VAP_FFN_STAMPS=1 python tools/stamps_ffn.py --rows 32000
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("VAP_FFN_STAMPS", "1")


def main():
    from voiceactivityprojection_amd import _native as N
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32000)
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    lib = N.lib()
    dev = torch.device("cuda", 0)
    M, D = args.rows, 256
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(M, D, generator=g).to(dev)
    ga, be = torch.ones(D, device=dev), torch.zeros(D, device=dev)
    W1 = (torch.randn(3 * D, D, generator=g) / 16).to(torch.bfloat16).to(dev)
    W2 = (torch.randn(D, 3 * D, generator=g) / 28).to(torch.bfloat16).to(dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    W1p, W2p = torch.empty_like(W1), torch.empty_like(W2)
    N.check(lib.vap_test_pack_weight(P(W1), P(W1p), 3 * D, D, st))
    N.check(lib.vap_test_pack_weight(P(W2), P(W2p), D, 3 * D, st))
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(args.iters):  # back to back, as in the engine
        N.check(lib.vap_test_ffn_packed(P(x), M, P(W1p), P(W2p), P(ga), P(be), st))
    ev1.record()
    torch.cuda.synchronize()
    print(f"event time per launch {ev0.elapsed_time(ev1) * 1e3 / args.iters:.2f} us")
    allb = np.zeros(8 * 24 + 2048, dtype=np.uint64)
    N.check(lib.vap_test_read_ffn_stamps(ctypes.c_void_p(allb.ctypes.data)))
    buf = allb[:192].reshape(8, 24)
    wall = allb[192:].reshape(1024, 2).astype(np.int64)
    nwg = (M + 63) // 64
    for i in range(8):
        if i * 64 >= nwg:
            break
        s = buf[i].astype(np.int64)
        print(f"wg{i*64}: total {s[21] - s[0]:6d} | ln {s[1] - s[0]:5d} bar {s[2] - s[1]:5d} | up "
              + " ".join(str(v) for v in np.diff(s[3:12])) + f" | gelu {s[12] - s[11]:5d} bar {s[13] - s[12]:5d} | down/4 "
              + " ".join(str(v) for v in np.diff(np.r_[s[13:20], s[20]])) + f" | drain {s[21] - s[20]:5d}")
    t0 = buf[:, 22].astype(np.int64)
    t1 = buf[:, 23].astype(np.int64)
    print("wall us per wg", ((t1 - t0) / 100).tolist())
    print("wall start us", ((t0 - t0.min()) / 100).tolist(), "end us", ((t1 - t0.min()) / 100).tolist())
    nw = min(nwg, 1024)
    ws, we = wall[:nw, 0], wall[:nw, 1]
    base = ws.min()
    print(f"all {nw} workgroups: first start 0, last start {(ws.max() - base) / 100:.2f} us, last end "
          f"{(we.max() - base) / 100:.2f} us, duration us min/median/max {np.min(we - ws) / 100:.2f} / "
          f"{np.median(we - ws) / 100:.2f} / {np.max(we - ws) / 100:.2f}")
    order = np.argsort(ws)
    print("start us by dispatch rank (every 32nd):", [round((ws[order[k]] - base) / 100, 2) for k in range(0, nw, 32)])
    print("slowest 8 (wg, start, dur):", [(int(k), round((ws[k] - base) / 100, 2), round((we[k] - ws[k]) / 100, 2))
                                        for k in np.argsort(we - ws)[-8:]])
    print("shader clock GHz", ((buf[:, 21].astype(np.int64) - buf[:, 0].astype(np.int64)) / ((t1 - t0) * 10.0)).round(2).tolist())


if __name__ == "__main__":
    main()
