#!/usr/bin/env python3
"""Per-phase k-step timing of the bf16 GEMM (gemm2) from in-kernel s_memtime stamps (GPU box).

    VAP_GEMM2_STAMPS=1 python tools/stamps_gemm.py [--case conv2]
"""
import argparse
import ctypes
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("VAP_GEMM2_STAMPS", "1")


def main():
    from voiceactivityprojection_amd import _native as N
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    lib = N.lib()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(2)
    S, rin, lda, K, Nn, M = 32, 16002, 512, 1024, 256, 8000  # conv2 of one chunk (mb_kernels conv2_plain)
    A = (torch.randn(S, rin, lda, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    W = (torch.randn(Nn, K, generator=g) / math.sqrt(K)).to(torch.bfloat16).to(dev)
    C = torch.empty(S, M, Nn, device=dev, dtype=torch.bfloat16)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    for _ in range(args.iters):
        N.check(lib.vap_test_gemm(1, P(A), lda, rin * lda, P(W), K, Nn, None, M, S, P(C), Nn, M * Nn, None, Nn,
                                  M * Nn, None, None, 0, 0, 0, st))
    torch.cuda.synchronize()
    allb = np.zeros(8 * 2 * 4 * 6 + 8 * 6, dtype=np.uint64)
    N.check(lib.vap_test_read_gemm_stamps(ctypes.c_void_p(allb.ctypes.data)))
    b = allb[:384].reshape(8, 2, 4, 6).astype(np.int64)
    tb = allb[384:].reshape(8, 6).astype(np.int64)
    print("tile phases (wave 0): [prologue DMA, k-loop, epilogue math, store issue, store drain | total]")
    for wg in range(8):
        t = tb[wg]
        print(f"wg{wg * 64:4d}: " + " ".join(f"{t[k + 1] - t[k]:6d}" for k in range(5)) + f" | {t[5] - t[0]:6d}")
    names = ["dma+frag", "->bar", "bar->", "mfma", "vmwait", "bar"]
    for wg in range(8):
        for h in range(2):
            rows = []
            for k in range(4):
                st6 = b[wg, h, k]
                nxt = b[wg, h, k + 1, 0] if k < 3 else st6[5]
                d = [st6[1] - st6[0], st6[2] - st6[1], st6[3] - st6[2], st6[4] - st6[3], st6[5] - st6[4]]
                rows.append(f"[{' '.join(f'{x:5d}' for x in d)} | step {nxt - st6[0] if k < 3 else 0:5d}]")
            print(f"wg{wg * 64:4d} wave{4 * h}: " + " ".join(rows))
    print("columns: frag-read, LOAD barrier wait, MFMA segment, DMA vmcnt wait, COMPUTE barrier wait | k-step total")


if __name__ == "__main__":
    main()
