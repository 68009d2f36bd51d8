"""conv2..4 kernel debug modes vs torch (GPU box): VAP_CONVK4_DBG=1 raw conv (no ChannelNorm / ReLU),
3 raw with G := 1 (sum of W per channel), 5 raw with W := 1 (sum of the input window per row)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from voiceactivityprojection_amd import _native as N  # noqa: E402

mode = int(os.environ.get("VAP_CONVK4_DBG", "1"))
S, L_in = int(sys.argv[1]) if len(sys.argv) > 1 else 1, int(sys.argv[2]) if len(sys.argv) > 2 else 520
g = torch.Generator().manual_seed(7)
L_out = (L_in + 2 - 4) // 2 + 1
x = torch.relu(torch.randn(S, L_in, 256, generator=g)).to(torch.bfloat16)
W = (torch.randn(256, 256, 4, generator=g) / 32).to(torch.bfloat16)
xp = torch.zeros(S, L_in + 2, 256, dtype=torch.bfloat16)
xp[:, 1:L_in + 1] = x
if mode == 1:
    ref = F.conv1d(x.float().transpose(1, 2), W.float(), None, stride=2, padding=1).transpose(1, 2)
elif mode == 3:
    ref = W.float().sum((1, 2))[None, None, :].expand(S, L_out, 256)
else:
    win = torch.stack([xp[:, 2 * t:2 * t + 4].float().sum((1, 2)) for t in range(L_out)], 1)
    ref = win[:, :, None].expand(S, L_out, 256)
wpk = W.permute(0, 2, 1).reshape(256, 1024).contiguous().cuda()
out = torch.zeros(S, L_out, 256, dtype=torch.bfloat16, device="cuda")
zd = torch.zeros(256).cuda()
od = torch.ones(256).cuda()
xd = xp.cuda()
st = torch.cuda.current_stream().cuda_stream
N.check(N.lib().vap_test_convk4(xd.data_ptr(), (L_in + 2) * 256, L_in + 2, wpk.data_ptr(), zd.data_ptr(),
                                od.data_ptr(), zd.data_ptr(), out.data_ptr(), L_out * 256, L_out, S, st))
torch.cuda.synchronize()
got = out.float().cpu()
err = (got - ref).abs()
print("mode", mode, "max err", round(err.max().item(), 4), "ref max", round(ref.abs().max().item(), 3))
e = err[0]
print("err by row//32:", [round(e[32 * r:32 * r + 32].max().item(), 3) for r in range((L_out + 31) // 32)])
print("err by ch//32:", [round(e[:, 32 * c:32 * c + 32].max().item(), 3) for c in range(8)])
print("err by row%32:", [round(e[r::32].max().item(), 2) for r in range(32)])
print("row0 got[:8]", [round(v, 3) for v in got[0, 0, :8].tolist()], "ref", [round(v, 3) for v in ref[0, 0, :8].tolist()])
print("row1 got[:8]", [round(v, 3) for v in got[0, 1, :8].tolist()], "ref", [round(v, 3) for v in ref[0, 1, :8].tolist()])
