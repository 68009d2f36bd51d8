"""Probe the lane layout of v_mfma_f32_16x16x4_f32 on the device (diagnostic)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from voiceactivityprojection_amd import _native as N
res = {}
for name in ("a_onehot", "b_onehot"):
    pass
out = {}
# A lane l = l (distinct values), B all ones -> D[i][j] = sum_k A[i][k]: reveals which lanes form a row
a = torch.arange(64, dtype=torch.float32, device="cuda") + 1
b = torch.ones(64, device="cuda")
d = torch.zeros(64, 4, device="cuda")
N.check(N.lib().vap_test_probe_mfma_f32(a.data_ptr(), b.data_ptr(), d.data_ptr(), torch.cuda.current_stream().cuda_stream))
torch.cuda.synchronize()
print("A=lane+1, B=1:\n", d.cpu().numpy().astype(int).tolist())
# one-hot A lane p, B = lane + 1 -> nonzero outputs show where lane p's A value lands and which B lanes pair
for p in (0, 1, 16, 17, 32):
    a = torch.zeros(64, device="cuda"); a[p] = 1
    b = torch.arange(64, dtype=torch.float32, device="cuda") + 1
    d.zero_()
    N.check(N.lib().vap_test_probe_mfma_f32(a.data_ptr(), b.data_ptr(), d.data_ptr(), torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    nz = [(l, r, int(v)) for l in range(64) for r in range(4) for v in [d[l, r].item()] if v != 0]
    print(f"A one-hot lane {p}: (out lane, reg, B lane+1) =", nz)
