"""First-forward vs later-forward difference: compares conv4 rows (LSTM input), the gate rows and the
LSTM output h between consecutive forwards of one model on the same input.  GPU box."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from voiceactivityprojection_amd import _native as N  # noqa: E402
from voiceactivityprojection_amd.weights import synthetic_state_dict, synthetic_waveform  # noqa: E402

from vap.model import VapGPT  # noqa: E402

m = VapGPT(precision="bf16")
m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0).items()}, strict=True)
m = m.to("cuda").eval()
B = int(os.environ.get("DB", "20"))
n = 320000
w = torch.from_numpy(np.stack([synthetic_waveform(300 + i, n) for i in range(B)])).cuda()
snaps = []
for call in range(3):
    m.forward(w)
    torch.cuda.synchronize()
    h = m._native(torch.device("cuda", 0))
    pl = (ctypes.c_int64 * 13)()
    N.check(N.lib().vap_test_plan(h, B, n, pl))
    X4, GX, H0, sh, s4 = pl[3], pl[4], pl[5], pl[12], pl[11]
    ws = m._ws
    S = 2 * B
    L4 = s4 // 256 - 2
    x4 = ws[X4:X4 + S * s4 * 2].view(torch.bfloat16).view(S, s4 // 256, 256).clone()
    gx = ws[GX:H0].clone()
    h0 = ws[H0:H0 + S * sh * 2].view(torch.bfloat16).view(S, sh // 256, 256).clone()
    snaps.append((x4, gx, h0))
    m.synchronize()
for a, b in ((0, 1), (1, 2), (0, 2)):
    x4a, gxa, h0a = snaps[a]
    x4b, gxb, h0b = snaps[b]
    print(f"calls {a} vs {b}: conv4 equal {torch.equal(x4a, x4b)}, gate rows equal {torch.equal(gxa, gxb)}")
    d = (h0a.float() - h0b.float()).abs()[:, 4:]  # [S][L4][256]
    for s in range(d.shape[0]):
        rows = torch.nonzero(d[s].amax(-1)).flatten()
        if len(rows):
            t0 = rows[0].item()
            units = torch.nonzero(d[s, t0]).flatten().tolist()
            print(f"  seq {s}: first differing step {t0}, units at it {units[:8]}.. ({len(units)}), max {d[s].max().item():.3g}")
    if not torch.equal(gxa, gxb):
        dd = torch.nonzero(gxa != gxb).flatten()
        print("  gate bytes differ:", len(dd), "first", dd[:4].tolist(), "last", dd[-4:].tolist())
