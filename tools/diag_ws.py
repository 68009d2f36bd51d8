"""Diagnostic: which workspace rows of sequence 0 differ between a large batch and the clip alone
(conv4 rows X4, gate rows GX, LSTM h rows H0, residual X)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vap.model import VapGPT  # noqa: E402
from voiceactivityprojection_amd import _native as N  # noqa: E402
from voiceactivityprojection_amd.weights import synthetic_state_dict  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 768
n = 40000
m = VapGPT(precision="bf16")
m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0).items()}, strict=True)
m = m.to("cuda").eval()
g = torch.Generator(device="cuda").manual_seed(5)
W = (0.1 * torch.randn(B, 2, n, device="cuda", generator=g)).clamp_(-1, 1)
L = N.frame_lengths(n)
D = 256


def snap(b):
    h = m._native(W.device)
    pl = (ctypes.c_int64 * 13)()
    N.check(N.lib().vap_test_plan(h, b, n, pl))
    ws = m._ws
    out = {}
    for name, off, stride, rows, width, dt in (("X4", pl[3], pl[11], L[4] + 2, D, torch.bfloat16),
                                               ("GX", pl[4], L[4] * 4 * D, L[4], 4 * D, torch.bfloat16),
                                               ("H0", pl[5], pl[12], L[4] + 4, D, torch.bfloat16)):
        es = 2
        nbytes = rows * width * es
        t = ws[off: off + nbytes].view(dt).view(rows, width).clone()
        out[name] = t
    return out


for rep in range(3):
    a = m(W[0:1])["logits"].clone()
    sa = snap(1)
    o = m(W[:B])["logits"].clone()
    m.synchronize()
    sb = snap(B)
    msg = []
    for k in sa:
        d = (sa[k].float() - sb[k].float()).abs().amax(-1)
        bad = d.nonzero().flatten()
        msg.append(f"{k}: {bad.numel()} rows differ, first {bad[:3].tolist()}")
    dl = (o[0] - a[0]).abs().amax(-1).nonzero().flatten()
    print(f"rep {rep}: logits first bad frame {dl[:1].tolist()} | " + " | ".join(msg), flush=True)
