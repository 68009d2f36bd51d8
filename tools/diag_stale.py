"""Diagnostic: is a large-batch error a read of stale rows (left by the previous call) or a wrong
computation?  Runs clip B-1 alone (its rows land where clip 0's go), then the batch twice."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vap.model import VapGPT  # noqa: E402
from voiceactivityprojection_amd.weights import synthetic_state_dict  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 768
n = 40000
m = VapGPT(precision="bf16")
m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0).items()}, strict=True)
m = m.to("cuda").eval()
g = torch.Generator(device="cuda").manual_seed(5)
W = (0.1 * torch.randn(B, 2, n, device="cuda", generator=g)).clamp_(-1, 1)
a0 = m(W[0:1])["logits"].clone()
for rep in range(3):
    m(W[B - 1:B])  # leaves clip B-1's rows in sequence slots 0/1
    o1 = m(W[:B])["logits"].clone()
    o2 = m(W[:B])["logits"].clone()
    m.synchronize()
    d1 = (o1[0] - a0[0]).abs().amax(-1)
    d2 = (o2[0] - a0[0]).abs().amax(-1)
    f1 = d1.nonzero().flatten()
    f2 = d2.nonzero().flatten()
    print(f"rep {rep}: after other clip: max {d1.max().item():.3g} first bad frame {f1[:1].tolist()} | "
          f"repeat: max {d2.max().item():.3g} first bad frame {f2[:1].tolist()}", flush=True)
