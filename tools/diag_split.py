"""Where do two forwards differ?  Same input through a fresh model and a used one, and split vs unsplit
back end (VAP_BE_SPLIT read per handle at creation): per output, max |diff| and the clips / frames
that differ.  GPU box."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from voiceactivityprojection_amd.weights import synthetic_state_dict, synthetic_waveform  # noqa: E402


def model():
    from vap.model import VapGPT
    m = VapGPT(precision="bf16")
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0).items()}, strict=True)
    return m.to("cuda").eval()


def batch(B, n, seed):
    return torch.from_numpy(np.stack([synthetic_waveform(seed + i, n) for i in range(B)])).cuda()


def cmp(tag, a, b):
    for k in ("logits", "vad", "probs"):
        if k not in a:
            continue
        d = (a[k].float() - b[k].float()).abs()
        if d.max().item() == 0:
            print(tag, k, "identical")
            continue
        dd = d.reshape(d.shape[0], d.shape[1], -1).amax(-1)  # [B][T]
        clips = torch.nonzero(dd.amax(1)).flatten().tolist()
        frames = torch.nonzero(dd.amax(0)).flatten().tolist()
        print(tag, k, "max", d.max().item(), "clips", clips[:40], "frames", frames[:5], "..", frames[-5:], len(frames))


B = int(os.environ.get("DB", "20"))
long = batch(B, 320000, 300)
short = batch(B, 40960, 340)
os.environ["VAP_BE_SPLIT"] = "1"
m1 = model()
r1 = m1.forward(long)
r1b = m1.forward(long)
torch.cuda.synchronize()
cmp("split1 repeat", r1, r1b)
os.environ["VAP_BE_SPLIT"] = "2"
m2 = model()
m2.forward(short)
r2 = m2.forward(long)
r2b = m2.forward(long)
m2.synchronize()
cmp("split2 repeat", r2, r2b)
cmp("split2 vs split1", r2, r1)
cmp("split2 second vs split1", r2b, r1)
