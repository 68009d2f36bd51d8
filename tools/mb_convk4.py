#!/usr/bin/env python3
"""conv2..4 kernel alone at the bench's conv2 shape (GPU box): ms per launch under HIP events.
VAP_CONVK4_DBG selects the debug mode (0 product, 1 raw conv, 3 G := 1 (no slab reads feed the
MFMAs), 5 W := 1); usage: python tools/mb_convk4.py [S] [L_in] [iters]."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from voiceactivityprojection_amd import _native as N  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 128
L_in = int(sys.argv[2]) if len(sys.argv) > 2 else 16000
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
L_out = (L_in + 2 - 4) // 2 + 1
x = torch.relu(torch.randn(S, L_in + 2, 256, device="cuda")).to(torch.bfloat16)
W = (torch.randn(256, 1024, device="cuda") / 32).to(torch.bfloat16)
b, g, be = torch.zeros(256, device="cuda"), torch.ones(256, device="cuda"), torch.zeros(256, device="cuda")
out = torch.empty(S, L_out, 256, dtype=torch.bfloat16, device="cuda")
st = torch.cuda.current_stream().cuda_stream


def run():
    N.check(N.lib().vap_test_convk4(x.data_ptr(), (L_in + 2) * 256, L_in + 2, W.data_ptr(), b.data_ptr(), g.data_ptr(),
                                    be.data_ptr(), out.data_ptr(), L_out * 256, L_out, S, st))


for _ in range(3):
    run()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(iters):
    run()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / iters
tiles = S * ((L_out + 255) // 256)
flop = 2.0 * S * L_out * 256 * 1024
print(f"convk4 dbg={os.environ.get('VAP_CONVK4_DBG', '0')} S={S} L_out={L_out}: {ms:.4f} ms, {flop / ms / 1e9:.1f} TF/s, "
      f"{tiles} tiles, {ms * 1e-3 * 2.4e9 / (tiles / 256):.0f} cycles per tile-round at 2.4 GHz")
