"""Batch-invariance sweep (diagnostic): logits of clip 0 / last clip at batch B vs the clip alone,
plus the encoder output (vap_encode) at the same B.  bf16 mode, 2.5 s clips unless --n."""
import argparse
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vap.model import VapGPT  # noqa: E402
from voiceactivityprojection_amd.weights import synthetic_state_dict  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=40000)
ap.add_argument("--bs", default="64,256,512,768,1000")
a = ap.parse_args()
m = VapGPT(precision="bf16")
m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0).items()}, strict=True)
m = m.to("cuda").eval()
g = torch.Generator(device="cuda").manual_seed(5)
Bmax = max(int(b) for b in a.bs.split(","))
W = (0.1 * torch.randn(Bmax, 2, a.n, device="cuda", generator=g)).clamp_(-1, 1)
alone = {}
for i in (0, Bmax - 1):
    alone[i] = (m(W[i:i + 1])["logits"].clone(), m.encode_audio(W[i:i + 1])[0].clone())
for B in (int(b) for b in a.bs.split(",")):
    out = m(W[:B])["logits"]
    enc = m.encode_audio(W[:B])[0]
    m.synchronize()
    res = []
    for i in (0, B - 1):
        if i not in alone:
            alone[i] = (m(W[i:i + 1])["logits"].clone(), m.encode_audio(W[i:i + 1])[0].clone())
        dl = (out[i] - alone[i][0][0]).abs().max().item()
        de = (enc[i] - alone[i][1][0]).abs().max().item()
        rows = (enc[i] - alone[i][1][0]).abs().amax(-1).nonzero()
        res.append(f"clip {i}: logits {dl:.3g} enc {de:.3g} enc rows bad {rows.numel()} first {rows[:3].flatten().tolist()}")
    print(f"B={B}: " + " | ".join(res), flush=True)
