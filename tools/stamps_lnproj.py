#!/usr/bin/env python3
"""Phase timing of the fused LN-projection kernel (k_block.hip lnproj) from s_memtime stamps (GPU box).

    python tools/stamps_lnproj.py --rows 32000 [--mode qkv_kvc|oproj_qc]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("VAP_LNPROJ_STAMPS", "1")


def main():
    from voiceactivityprojection_amd import _native as N
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32000)
    ap.add_argument("--mode", default="qkv_kvc")
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    lib = N.lib()
    dev = torch.device("cuda", 0)
    M, D = args.rows, 256
    oproj = args.mode == "oproj_qc"
    np_, nr = (1, 0) if oproj else (3, 2)
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(M, D, generator=g).to(dev)
    O = torch.randn(M, D, generator=g).to(torch.bfloat16).to(dev)
    ga, be = torch.ones(D, device=dev), torch.zeros(D, device=dev)
    Wo = (torch.randn(D, D, generator=g) / 16).to(torch.bfloat16).to(dev)
    Wp = (torch.randn(np_ * D, D, generator=g) / 16).to(torch.bfloat16).to(dev)
    Wr = (torch.randn(2 * D, D, generator=g) / 16).to(torch.bfloat16).to(dev)
    cp = torch.empty(M, np_ * D, dtype=torch.bfloat16, device=dev)
    cr = torch.empty(M, 2 * D, dtype=torch.bfloat16, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(args.iters):
        N.check(lib.vap_test_lnproj(P(x), P(O) if oproj else None, M, P(Wo) if oproj else None, P(Wp), np_,
                                    P(Wr) if nr else None, nr, P(cp), P(cr) if nr else None, P(ga), P(be), st))
    ev1.record()
    torch.cuda.synchronize()
    print(f"event time per call (incl. weight packing + sync) {ev0.elapsed_time(ev1) * 1e3 / args.iters:.2f} us")
    buf = np.zeros(8 * 24, dtype=np.uint64)
    N.check(lib.vap_test_read_lnproj_stamps(ctypes.c_void_p(buf.ctypes.data)))
    buf = buf.reshape(8, 24).astype(np.int64)
    npass = np_ + nr
    for i in range(8):
        s = buf[i]
        if s[0] == 0:
            continue
        pre = (f"opanel {s[1] - s[0]:5d} oproj {s[2] - s[1]:5d} ln {s[3] - s[2]:5d}" if oproj
               else f"load+ln {s[3] - s[0]:5d}")
        passes = " | ".join(f"mma {s[4 + p] - (s[3] if p == 0 else s[10 + p - 1]):5d} st {s[10 + p] - s[4 + p]:5d}"
                            for p in range(npass))
        print(f"wg{i*64}: total {s[16] - s[0]:6d} | {pre} | {passes} | drain {s[16] - s[10 + npass - 1]:5d}")


if __name__ == "__main__":
    main()
