"""Diagnostic: the resident LSTM with every sequence fed the SAME gate rows must give the same h for
every sequence; counts sequences that differ from sequence 0 at several S, alone and beside a
concurrent matmul stream."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from voiceactivityprojection_amd import _native as N  # noqa: E402

lib = N.lib()
dev = torch.device("cuda", 0)
g = torch.Generator(device="cpu").manual_seed(0)
T = 250
gx0 = (torch.randn(1, T, 1024, generator=g) * 0.5).to(torch.bfloat16).to(dev)
whh = (torch.randn(1024, 256, generator=g) / 16).to(dev)
whp = torch.empty(1024 * 256, dtype=torch.bfloat16, device=dev)
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
side = torch.cuda.Stream()
a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
for S in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "128,1024,1280,1536,2048,4096").split(",")]:
    gx = gx0.expand(S, T, 1024).contiguous()
    for busy in (False, True):
        out = torch.zeros(S, T, 256, dtype=torch.bfloat16, device=dev)
        if busy:
            with torch.cuda.stream(side):
                for _ in range(20):
                    a = (a @ a).clamp_(-1, 1)
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        N.check(lib.vap_test_lstm(1, P(gx), S, T, P(whh), P(whp), P(out), 2, st))
        torch.cuda.synchronize()
        d = (out.float() - out[:1].float()).abs().amax(-1)  # [S][T]
        bad = (d.amax(-1) > 0).nonzero().flatten()
        first = [int((d[s] > 0).nonzero()[0]) for s in bad[:4].tolist()]
        print(f"S={S} busy={busy}: {bad.numel()} sequences differ from seq 0; e.g. {bad[:4].tolist()} first bad step {first}",
              flush=True)
