"""Diagnostic: resident bf16 LSTM vs torch, locating mismatches (GPU box)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from voiceactivityprojection_amd import _native as N

def run(S, T, variant, seed=3):
    g = torch.Generator().manual_seed(seed)
    gx = torch.randn(S, T, 1024, generator=g).to(torch.bfloat16)
    whh = (torch.rand(1024, 256, generator=g) * 2 - 1) / 16
    out = torch.zeros(S, T, 256, device="cuda", dtype=torch.bfloat16)
    packed = torch.zeros(1024 * 256, device="cuda", dtype=torch.bfloat16)
    gxd = gx.cuda() if variant == 0 else gx.float().cuda()
    whd = whh.cuda()
    N.check(N.lib().vap_test_lstm(1, gxd.data_ptr(), S, T, whd.data_ptr(), packed.data_ptr(), out.data_ptr(), variant,
                                  torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    wr = whh.to(torch.bfloat16).float()
    h = torch.zeros(S, 256); c = torch.zeros(S, 256); ys = []
    for t in range(T):
        z = gx[:, t].float() + h.to(torch.bfloat16).float() @ wr.T
        i, f, gg, o = z.split(256, -1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        h = torch.sigmoid(o) * torch.tanh(c); ys.append(h)
    ref = torch.stack(ys, 1)
    o = out.float().cpu()
    err = (o - ref).abs()
    print(f"S={S} T={T} variant={variant}: max err {err.max().item():.4g}, nonfinite {(~torch.isfinite(o)).sum().item()}")
    bad = (err > 0.05) | ~torch.isfinite(o)
    if bad.any():
        idx = bad.nonzero()
        print("  first bad (s,t,u):", idx[:8].tolist(), "count", idx.shape[0])
        print("  bad seqs:", sorted(set(idx[:, 0].tolist()))[:20], " bad t min:", idx[:, 1].min().item(),
              " units:", sorted(set((idx[:, 2] // 16).tolist()))[:20])
        s, t, u = idx[0].tolist()
        print("  got", o[s, t, u].item(), "ref", ref[s, t, u].item())

for S, T in ((16, 5), (16, 37), (20, 37), (4, 37), (32, 3)):
    run(S, T, 0)
run(20, 37, 1)
