#!/usr/bin/env python3
"""Per-k-step timing of the row-panel kernel from in-kernel s_memtime stamps (GPU box).

    VAP_RP_STAMPS=1 [VAP_RP_V1=1] python tools/stamps_rowpanel.py --rows 32000 --epi 0

Wave 0 of 8 sampled workgroups: panel load, each k-step (24 for N = 768), each N tile's stores,
final store drain.  Cycle deltas of the shader clock.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("VAP_RP_STAMPS", "1")


def main():
    from voiceactivityprojection_amd import _native as N
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32000)
    ap.add_argument("--epi", type=int, default=0)
    args = ap.parse_args()
    lib = N.lib()
    dev = torch.device("cuda", 0)
    M, D, NN = args.rows, 256, 768
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(M, D, generator=g).to(dev)
    ga = torch.ones(D, device=dev)
    be = torch.zeros(D, device=dev)
    W = (torch.randn(NN, D, generator=g) / 16).to(torch.bfloat16).to(dev)
    C = torch.empty(M, NN, device=dev, dtype=torch.bfloat16)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    for _ in range(5):
        N.check(lib.vap_test_rowpanel(P(x), D, M, P(W), D, NN, P(C), NN, None, P(ga), P(be), 1, args.epi, st))
    torch.cuda.synchronize()
    buf = np.zeros((8, 32), dtype=np.uint64)
    N.check(lib.vap_test_read_rp_stamps(ctypes.c_void_p(buf.ctypes.data)))
    nwg = (M + 63) // 64
    for i in range(8):
        if i * 64 >= nwg:
            break
        s = buf[i].astype(np.int64)
        ks = np.diff(s[2:26])
        print(f"wg{i*64}: total {s[29] - s[0]:6d} | panel {s[1] - s[0]:5d} | ksteps " + " ".join(str(v) for v in ks)
              + f" | last-step->tile2 stores {s[28] - s[25]:5d} | drain {s[29] - s[28]:5d}")
    rel = buf[:, 0].astype(np.int64)
    print("start offsets", (rel - rel.min()).tolist())


if __name__ == "__main__":
    main()
