"""Diagnose the quad-split fp32 recurrence (test ABI variant 4) against a torch fp32 LSTM: error per step
and per unit quarter."""
import sys, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from voiceactivityprojection_amd import _native as N

g = torch.Generator().manual_seed(3)
S, T = int(sys.argv[1]) if len(sys.argv) > 1 else 16, int(sys.argv[2]) if len(sys.argv) > 2 else 4
gx = torch.randn(S, T, 1024, generator=g)
whh = (torch.rand(1024, 256, generator=g) * 2 - 1) / 16
out = torch.zeros(S, T, 256, device="cuda")
packed = torch.zeros(1024 * 256, device="cuda")
N.check(N.lib().vap_test_lstm(0, gx.cuda().data_ptr(), S, T, whh.cuda().data_ptr(), packed.data_ptr(), out.data_ptr(), 4,
                              torch.cuda.current_stream().cuda_stream))
torch.cuda.synchronize()
h = torch.zeros(S, 256); c = torch.zeros(S, 256); ys = []
for t in range(T):
    z = gx[:, t] + h @ whh.T
    i, f, gg, o = z.split(256, -1)
    c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
    h = torch.sigmoid(o) * torch.tanh(c)
    ys.append(h)
ref = torch.stack(ys, 1)
got = out.cpu()
for t in range(T):
    e = (got[:, t] - ref[:, t]).abs()
    print(t, "max", float(e.max()), "per quarter", [float(e[:, 64 * q:64 * q + 64].max()) for q in range(4)],
          "per wave of q0", [float(e[:, 16 * w:16 * w + 16].max()) for w in range(4)])
e = (got[:, 1] - ref[:, 1]).abs()
print("step1 seq0 units with err>1e-3:", (e[0] > 1e-3).nonzero().flatten().tolist()[:64])
