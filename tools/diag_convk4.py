"""Error pattern of the conv2..4 kernel vs torch (GPU box): which rows / channels disagree."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from voiceactivityprojection_amd import _native as N  # noqa: E402

S, L_in = 1, 520
g = torch.Generator().manual_seed(7)
L_out = (L_in + 2 - 4) // 2 + 1
x = torch.relu(torch.randn(S, L_in, 256, generator=g)).to(torch.bfloat16)
W = (torch.randn(256, 256, 4, generator=g) / 32).to(torch.bfloat16)
zero = torch.zeros(256)
one = torch.ones(256)
mode = sys.argv[1] if len(sys.argv) > 1 else "full"
if mode.startswith("tap"):  # only tap K nonzero (tapKcbC: and only input channel block C)
    k = int(mode[3])
    if "cb" in mode:
        cb = int(mode.split("cb")[1])
        keep = torch.zeros(256, dtype=torch.bool)
        keep[32 * cb:32 * cb + 32] = True
        W[:, ~keep, :] = 0
    for j in range(4):
        if j != k:
            W[:, :, j] = 0
ref = F.conv1d(x.float().transpose(1, 2), W.float(), None, stride=2, padding=1).transpose(1, 2)
xp = torch.zeros(S, L_in + 2, 256, dtype=torch.bfloat16)
xp[:, 1:L_in + 1] = x
wpk = W.permute(0, 2, 1).reshape(256, 1024).contiguous().cuda()
out = torch.zeros(S, L_out, 256, dtype=torch.bfloat16, device="cuda")
st = torch.cuda.current_stream().cuda_stream
# gamma = 1, beta = 0, bias 0: output = relu(CN(conv)); compare CN'd reference
mu, var = ref.mean(-1, keepdim=True), ref.var(-1, keepdim=True)
refn = torch.relu((ref - mu) * torch.rsqrt(var + 1e-5))
xd, zd, od = xp.cuda(), zero.cuda(), one.cuda()  # named: temporaries would be freed and reused
N.check(N.lib().vap_test_convk4(xd.data_ptr(), (L_in + 2) * 256, L_in + 2, wpk.data_ptr(), zd.data_ptr(),
                                od.data_ptr(), zd.data_ptr(), out.data_ptr(), L_out * 256, L_out, S, st))
torch.cuda.synchronize()
got = out.float().cpu()
err = (got - refn).abs()[0]
print("max err", err.max().item(), "rows", L_out)
print("err by row%32:", [round(err[r::32].max().item(), 2) for r in range(32)])
print("err by ch%32:", [round(err[:, c::32].max().item(), 2) for c in range(32)])
print("err by ch//32:", [round(err[:, 32 * c:32 * c + 32].max().item(), 2) for c in range(8)])
print("err by row//32:", [round(err[32 * r:32 * r + 32].max().item(), 2) for r in range((L_out + 31) // 32)])
# try to find a permutation: for row 5, which reference channel matches got channel c
r = 5
for c in (0, 1, 4, 8, 16):
    d = (refn[0, r] - got[0, r, c]).abs()
    print("row", r, "got ch", c, got[0, r, c].item(), "best ref ch", int(d.argmin()), "ref same ch", refn[0, r, c].item())
print("got: frac zero", (got == 0).float().mean().item(), "mean", got.mean().item(), "ref frac zero", (refn == 0).float().mean().item())
print("got row 5 first 16:", got[0, 5, :16].tolist())
print("ref row 5 first 16:", [round(v, 3) for v in refn[0, 5, :16].tolist()])
dbg = int(os.environ.get("VAP_CONVK4_DBG", "0"))
if dbg & 1:
    r2 = ref.clone()
    if dbg & 2:
        r2 = W.float().sum(dim=(1, 2))[None, None, :].expand(S, L_out, 256) * 1.0
    if dbg & 4:
        r2 = F.conv1d(x.float().transpose(1, 2), torch.ones(256, 256, 4), None, stride=2, padding=1).transpose(1, 2)
    e = (got - r2).abs()[0]
    print("raw: max err", e.max().item(), "got[5,:8]", got[0, 5, :8].tolist(), "ref[5,:8]", [round(v, 3) for v in r2[0, 5, :8].tolist()])
    print("raw err by row//32:", [round(e[32 * r:32 * r + 32].max().item(), 2) for r in range((L_out + 31) // 32)])
if dbg & 1:
    print("raw err rows 0..35:", [round(e[r].max().item(), 2) for r in range(36)])
    print("raw err row 0..31 by ch//32:", [round(e[:32, 32 * c:32 * c + 32].max().item(), 2) for c in range(8)])
if dbg == 1 and mode.startswith("tap"):
    k = int(mode[3])
    cands = {"zero": torch.zeros(256)}
    for r in range(0, 8):
        cands[f"buf{r}"] = xp[0, r].float()
    cands["last"] = xp[0, -1].float()
    for name, v in cands.items():
        pred = W[:, :, k].float() @ v
        print("row0 candidate", name, "err", (got[0, 0] - pred).abs().max().item())
