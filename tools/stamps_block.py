#!/usr/bin/env python3
"""Phase timing of the fused layer-tail kernel (k_block.hip) from in-kernel s_memtime stamps (GPU box).

    python tools/stamps_block.py --rows 32000 [--cus 248]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("VAP_BLOCK_STAMPS", "1")


def main():
    from voiceactivityprojection_amd import _native as N
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32000)
    ap.add_argument("--cus", type=int, default=248)
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    lib = N.lib()
    dev = torch.device("cuda", 0)
    M, D = args.rows, 256
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(M, D, generator=g).to(dev)
    O = torch.randn(M, D, generator=g).to(torch.bfloat16).to(dev)
    ga, be = torch.ones(D, device=dev), torch.zeros(D, device=dev)
    Wo = (torch.randn(D, D, generator=g) / 16).to(torch.bfloat16).to(dev)
    W1 = (torch.randn(3 * D, D, generator=g) / 16).to(torch.bfloat16).to(dev)
    W2 = (torch.randn(D, 3 * D, generator=g) / 28).to(torch.bfloat16).to(dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    pk = []
    for W in (Wo, W1, W2):
        Wp = torch.empty_like(W)
        N.check(lib.vap_test_pack_weight(P(W), P(Wp), W.shape[0], W.shape[1], st))
        pk.append(Wp)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(args.iters):
        N.check(lib.vap_test_block_packed(P(x), P(O), M, P(pk[0]), P(pk[1]), P(pk[2]), P(ga), P(be), args.cus, st))
    ev1.record()
    torch.cuda.synchronize()
    print(f"event time per launch {ev0.elapsed_time(ev1) * 1e3 / args.iters:.2f} us")
    buf = np.zeros(8 * 24, dtype=np.uint64)
    N.check(lib.vap_test_read_block_stamps(ctypes.c_void_p(buf.ctypes.data)))
    buf = buf.reshape(8, 24).astype(np.int64)
    for i in range(8):
        s = buf[i]
        if s[0] == 0:
            continue
        sl = " | ".join(f"up {s[4+4*k] - s[3+4*k if k == 0 else 3+4*k]:5d} gelu+bar {s[5+4*k] - s[4+4*k]:5d} "
                        f"hw+bar {s[6+4*k] - s[5+4*k]:5d} down {s[7+4*k] - s[6+4*k]:5d}" for k in range(3))
        print(f"wg{i*32}: total {s[17] - s[0]:6d} | opanel {s[1] - s[0]:5d} oproj {s[2] - s[1]:5d} ln {s[3] - s[2]:5d} | "
              + sl + f" | store {s[16] - s[15]:5d} drain {s[17] - s[16]:5d}")


if __name__ == "__main__":
    main()
