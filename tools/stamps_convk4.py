#!/usr/bin/env python3
"""Phase stamps of the conv2..4 kernel at the bench's conv2 shape (GPU box):
start | 8 x (block barrier passed) | k-loop done | stores issued | stores drained."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["VAP_CONVK4_DBG"] = "16"
from voiceactivityprojection_amd import _native as N  # noqa: E402

S, L_in = int(sys.argv[1]) if len(sys.argv) > 1 else 128, int(sys.argv[2]) if len(sys.argv) > 2 else 16000
L_out = (L_in + 2 - 4) // 2 + 1
x = torch.relu(torch.randn(S, L_in + 2, 256, device="cuda")).to(torch.bfloat16)
W = (torch.randn(256, 1024, device="cuda") / 32).to(torch.bfloat16)
b, g, be = torch.zeros(256, device="cuda"), torch.ones(256, device="cuda"), torch.zeros(256, device="cuda")
out = torch.empty(S, L_out, 256, dtype=torch.bfloat16, device="cuda")
host = np.zeros(8 * 14, dtype=np.uint64)
N.check(N.lib().vap_test_convk4_stamps(ctypes.c_void_p(host.ctypes.data)))
st = torch.cuda.current_stream().cuda_stream
for _ in range(int(os.environ.get('REPS', '3'))):
    N.check(N.lib().vap_test_convk4(x.data_ptr(), (L_in + 2) * 256, L_in + 2, W.data_ptr(), b.data_ptr(), g.data_ptr(),
                                    be.data_ptr(), out.data_ptr(), L_out * 256, L_out, S, st))
names = ["pro+b0"] + [f"b{i}" for i in range(1, 8)] + ["b7end", "epi_math+issue", "drain"]
h = host.reshape(8, 14).astype(np.int64)
for wg in range(8):
    d = np.diff(h[wg, :12])
    ghz = (h[wg, 11] - h[wg, 0]) / max(1, h[wg, 13] - h[wg, 12]) * 0.1
    print(f"wg{wg}: total {h[wg, 11] - h[wg, 0]:7d} | " + " ".join(f"{n}={v}" for n, v in zip(names, d)) + f" | clock {ghz:.2f} GHz")
