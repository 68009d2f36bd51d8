"""Kernel-level numerics: each HIP kernel (through the kernel test ABI of libvap_hip.so) against a
plain PyTorch fp32 reference of the same op.  fp32 storage mode must agree to ~1e-5 relative
(exact fp32 MFMA); bf16 storage mode is checked against the reference evaluated on the SAME
bf16-rounded inputs (fp32 accumulate), so the tolerance only covers accumulation order and the
bf16 rounding of the output."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

PREC = {"fp32": (0, torch.float32), "bf16": (1, torch.bfloat16), "split": (2, torch.float32)}


def lib():
    from voiceactivityprojection_amd import _native as N

    return N


def _st():
    return torch.cuda.current_stream().cuda_stream


def _run(fn, *args):
    N = lib()
    N.check(fn(*args), fn.__name__)
    torch.cuda.synchronize()


def _p(t):
    return t.data_ptr() if t is not None else None


@pytest.mark.parametrize("prec", ["fp32", "bf16", "split"])
@pytest.mark.parametrize("case", ["plain", "conv_cn_relu", "resid", "ln_gelu", "gelu", "comb", "many_tiles",
                                  "many_tiles_n1024"])
def test_gemm(prec, case):
    """Implicit-conv GEMM with every epilogue form.  comb = act(LN(A W)) + residual (the combinator's
    second half); many_tiles* = more 256-row tiles than CUs, so persistent workgroups walk several
    tiles with the DMA stream running across the tile seams (N 256 and N 1024).  split = the fp32 parity
    mode's kernel (fp32 operands as hi + lo bf16 pairs, three bf16 MFMAs per tile-step): fp32 accuracy
    to ~2^-16 of a product, checked at 3e-5 of the output scale."""
    N = lib()
    code, dt = PREC[prec]
    g = torch.Generator().manual_seed(1)
    if case == "plain":
        S, Mps, K, Nn, lda = 1, 300, 256, 768, 256
    elif case == "conv_cn_relu":
        S, Mps, K, Nn, lda = 3, 77, 1024, 256, 512
    elif case in ("resid", "gelu"):
        S, Mps, K, Nn, lda = 2, 130, 768, 256, 768
    elif case == "comb":
        S, Mps, K, Nn, lda = 2, 300, 256, 256, 256
    elif case == "many_tiles":
        S, Mps, K, Nn, lda = 2, 40000, 256, 256, 256
    elif case == "many_tiles_n1024":
        S, Mps, K, Nn, lda = 1, 20000, 256, 1024, 256
    else:
        S, Mps, K, Nn, lda = 2, 201, 1280, 256, 512
    L = (Mps - 1) * lda + K
    A_flat = torch.randn(S, L, generator=g)
    W = torch.randn(Nn, K, generator=g) / math.sqrt(K)
    bias = torch.randn(Nn, generator=g) * 0.1
    gamma = 1 + 0.2 * torch.randn(Nn, generator=g)
    beta = 0.1 * torch.randn(Nn, generator=g)
    add = torch.randn(S, Mps, Nn, generator=g)
    Aq = A_flat.to(dt)
    Wq = W.to(dt)
    # reference on the (rounded) inputs
    Ar, Wr = Aq.float(), Wq.float()
    idx = torch.arange(Mps)[:, None] * lda + torch.arange(K)[None, :]
    X = Ar[:, idx]  # (S, Mps, K) overlapping rows
    ref = X @ Wr.T
    norm = act = 0
    use_bias = case not in ("plain", "comb", "many_tiles")
    use_add = case in ("resid", "comb")
    if use_bias:
        ref = ref + bias
    if case == "conv_cn_relu":
        norm, act = 1, 1
        mu = ref.mean(-1, keepdim=True)
        var = ref.var(-1, keepdim=True)
        ref = torch.relu((ref - mu) * torch.rsqrt(var + 1e-5) * gamma + beta)
    elif case in ("ln_gelu", "comb"):
        norm, act = 2, 2
        ref = F.gelu(F.layer_norm(ref, (Nn,), gamma, beta))
    elif case == "gelu":
        act = 2
        ref = F.gelu(ref)
    if use_add:
        ref = ref + add
    out_f32 = 1 if (prec != "bf16" or case in ("resid", "ln_gelu", "comb")) else 0
    C = torch.zeros(S, Mps, Nn, device="cuda", dtype=torch.float32 if out_f32 else dt)
    Ad, Wd = Aq.cuda(), Wq.cuda()
    bd, gd, bed, addd = bias.cuda(), gamma.cuda(), beta.cuda(), add.cuda()
    _run(N.lib().vap_test_gemm, code, _p(Ad), lda, A_flat.shape[1], _p(Wd), K, Nn, _p(bd) if use_bias else None,
         Mps, S, _p(C), Nn, Mps * Nn, _p(addd) if use_add else None, Nn, Mps * Nn, _p(gd), _p(bed), norm, act,
         out_f32, _st())
    got = C.float().cpu()
    tol = {"fp32": 2e-4, "split": 3e-5}.get(prec, 1e-2 if not out_f32 else 3e-3)
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= tol * max(1.0, scale), f"{prec}/{case}: max err {err} (scale {scale})"


@pytest.mark.parametrize("S,L_in,a,b", [(3, 160, 0, -1), (2, 1601, 0, -1), (2, 1600, 37, 301), (1, 514, 1, 257),
                                         (4, 6000, 1000, -1)])
def test_convk4(S, L_in, a, b):
    """CPC conv2..4 kernel (k_conv234.hip): k4 s2 p1 conv + bias + ChannelNorm (unbiased) + ReLU on a
    padded [S][L_in + 2][256] bf16 activation (one zero pad row in front and behind), output rows
    [a, b) of the layer, against torch conv1d on the same bf16 inputs (encoder_components.py:87-103)."""
    N = lib()
    g = torch.Generator().manual_seed(7)
    L_out = (L_in + 2 - 4) // 2 + 1
    b = L_out if b < 0 else b
    M = b - a
    x = torch.relu(torch.randn(S, L_in, 256, generator=g)).to(torch.bfloat16)
    W = (torch.randn(256, 256, 4, generator=g) / 32).to(torch.bfloat16)  # [out][in][tap]
    bias = torch.randn(256, generator=g) * 0.1
    gamma = 1 + 0.2 * torch.randn(256, generator=g)
    beta = 0.1 * torch.randn(256, generator=g)
    ref = F.conv1d(x.float().transpose(1, 2), W.float(), bias, stride=2, padding=1).transpose(1, 2)[:, a:b]
    mu, var = ref.mean(-1, keepdim=True), ref.var(-1, keepdim=True)
    ref = torch.relu((ref - mu) * torch.rsqrt(var + 1e-5) * gamma + beta)
    xp = torch.zeros(S, L_in + 2, 256, dtype=torch.bfloat16)
    xp[:, 1:L_in + 1] = x
    xd = xp.cuda()
    wpk = W.permute(0, 2, 1).reshape(256, 1024).contiguous().cuda()  # [n][tap * 256 + ci]
    out = torch.full((S, M + 3, 256), 7.0, dtype=torch.bfloat16, device="cuda")
    in_off = 2 * a * 256 * 2
    bd, gd, bed = bias.cuda(), gamma.cuda(), beta.cuda()  # named: temporaries would be freed and reused
    _run(N.lib().vap_test_convk4, xd.data_ptr() + in_off, (L_in + 2) * 256, L_in + 2 - 2 * a, _p(wpk),
         _p(bd), _p(gd), _p(bed), _p(out), (M + 3) * 256, M, S, _st())
    got = out.float().cpu()
    err = (got[:, :M] - ref).abs().max().item()
    assert err <= 3e-2 * max(1.0, ref.abs().max().item()), f"max err {err}"
    assert bool((got[:, M:] == 7.0).all()), "rows past M were written"  # the tile's store guard
    assert torch.all(got[:, M:] == 7.0), "rows past the range were written"


@pytest.mark.parametrize("prec", ["fp32", "bf16", "split"])
@pytest.mark.parametrize("kv_swap", [0, 1])
def test_attention(prec, kv_swap):
    N = lib()
    code, dt = PREC[prec]
    g = torch.Generator().manual_seed(2)
    S, T, H, D = 4, 150, 4, 256
    Q = torch.randn(S, T, D, generator=g).to(dt)
    K = torch.randn(S, T, D, generator=g).to(dt)
    V = torch.randn(S, T, D, generator=g).to(dt)
    slopes = torch.tensor([0.25, 0.0625, 0.015625, 0.00390625])
    scale = 1 / 16
    O = torch.zeros(S, T, D, device="cuda", dtype=dt)
    Qd, Kd, Vd, sd = Q.cuda(), K.cuda(), V.cuda(), slopes.cuda()
    _run(N.lib().vap_test_attention, code, _p(Qd), D, T * D, _p(Kd), D, T * D, _p(Vd), D, T * D, _p(O), D, T * D,
         _p(sd), S, T, H, kv_swap, scale, _st())
    kv = [(s ^ 1) if kv_swap else s for s in range(S)]  # cross: other speaker of the clip
    q = Q.float().view(S, T, H, 64).transpose(1, 2)
    k = K.float()[kv].view(S, T, H, 64).transpose(1, 2)
    v = V.float()[kv].view(S, T, H, 64).transpose(1, 2)
    att = torch.einsum("bhid,bhjd->bhij", q, k) * scale
    bias = torch.arange(T).float().view(1, 1, 1, -1) * slopes.view(1, -1, 1, 1)
    mask = torch.tril(torch.ones(T, T)) == 0
    att = (att + bias).masked_fill(mask, float("-inf")).softmax(-1)
    ref = (att @ v).transpose(1, 2).reshape(S, T, D)
    err = (O.float().cpu() - ref).abs().max().item()
    tol = {"fp32": 2e-5, "split": 5e-5}.get(prec, 2e-2)
    assert err <= tol, f"{prec}: attention max err {err}"


@pytest.mark.parametrize("prec,variant,S", [("fp32", 0, 20), ("bf16", 0, 20), ("bf16", 1, 20), ("bf16", 2, 20),
                                            ("bf16", 3, 20), ("bf16", 3, 300), ("bf16", 5, 20), ("bf16", 5, 300),
                                            ("fp32", 4, 20), ("fp32", 4, 300)])
def test_lstm(prec, variant, S):
    """variant 0 = the resident kernel for that precision (bf16: W_hh resident in AGPR/VGPR/LDS,
    bf16 gx); variant 1 = the L2-streaming kernel in bf16 (fp32 gx); variant 2 = the resident bf16
    path with gate scales folded into W_hh and gx (the ABI scales gx), exp2-domain cell; variant 3 =
    the engine's default: W_hh split over workgroup pairs that exchange h halves every step (S = 300:
    19 pairs, a padding pair in the last 16-block group); variant 5 = the same operands on workgroup quads
    (lstm_quadb_kernel, VAP_LSTM_QUAD); fp32 variant 4 = the parity mode's default: W_hh
    split over workgroup quads, split-bf16 products, fp32 gates / state / h (S = 300: 19 quads, padding
    quads in the last 32-block group)."""
    N = lib()
    code, dt = PREC[prec]
    g = torch.Generator().manual_seed(3)
    T = 37
    gx = torch.randn(S, T, 1024, generator=g)
    if prec == "bf16" and variant in (0, 2, 3, 5):
        gx = gx.to(torch.bfloat16).float()
    whh = (torch.rand(1024, 256, generator=g) * 2 - 1) / 16
    out = torch.zeros(S, T, 256, device="cuda", dtype=dt)
    packed = torch.zeros(1024 * 256, device="cuda", dtype=dt)
    gxd = gx.cuda().to(torch.bfloat16) if (prec == "bf16" and variant in (0, 2, 3, 5)) else gx.cuda()
    whd = whh.cuda()
    _run(N.lib().vap_test_lstm, code, _p(gxd), S, T, _p(whd), _p(packed), _p(out), variant, _st())
    wr = whh.to(dt).float()
    h = torch.zeros(S, 256)
    c = torch.zeros(S, 256)
    ys = []
    for t in range(T):
        z = gx[:, t] + h.to(dt).float() @ wr.T
        i, f, gg, o = z.split(256, -1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        h = torch.sigmoid(o) * torch.tanh(c)
        ys.append(h)
    ref = torch.stack(ys, 1)
    err = (out.float().cpu() - ref).abs().max().item()
    tol = 2e-5 if prec == "fp32" else 1e-2
    assert err <= tol, f"{prec}/{variant}: lstm max err {err}"


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_conv0(prec):
    N = lib()
    code, dt = PREC[prec]
    g = torch.Generator().manual_seed(4)
    B, n = 2, 3001
    wav = torch.randn(B, 2, n, generator=g) * 0.1
    w0 = torch.randn(256, 1, 10, generator=g) / math.sqrt(10)
    b0 = torch.randn(256, generator=g) * 0.1
    ga = 1 + 0.2 * torch.randn(256, generator=g)
    be = 0.1 * torch.randn(256, generator=g)
    L0 = (n + 6 - 10) // 5 + 1
    out = torch.zeros(2 * B, L0 + 4, 256, device="cuda", dtype=dt)
    d = [t.cuda() for t in (wav, w0, b0, ga, be)]
    _run(N.lib().vap_test_conv0, code, _p(d[0]), B, n, L0, _p(d[1]), _p(d[2]), _p(d[3]), _p(d[4]), _p(out), _st())
    x = wav.reshape(2 * B, 1, n)  # clip-major sequences (seq = 2*clip + channel)
    y = F.conv1d(x, w0, b0, stride=5, padding=3)
    mu, var = y.mean(1, keepdim=True), y.var(1, keepdim=True)
    y = torch.relu((y - mu) * torch.rsqrt(var + 1e-5) * ga.view(1, -1, 1) + be.view(1, -1, 1)).transpose(1, 2)
    got = out.float().cpu()[:, 2:L0 + 2]
    err = (got - y).abs().max().item()
    tol = 2e-5 if prec == "fp32" else 2e-2
    assert err <= tol, f"{prec}: conv0 max err {err}"


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_layernorm(prec):
    N = lib()
    code, dt = PREC[prec]
    g = torch.Generator().manual_seed(5)
    x = torch.randn(77, 256, generator=g) * 3 + 1
    ga = 1 + 0.2 * torch.randn(256, generator=g)
    be = 0.1 * torch.randn(256, generator=g)
    out = torch.zeros(77, 256, device="cuda", dtype=dt)
    raw = torch.zeros(77, 256, device="cuda", dtype=dt)
    d = [t.cuda() for t in (x, ga, be)]
    _run(N.lib().vap_test_layernorm, code, _p(d[0]), 77, _p(d[1]), _p(d[2]), _p(out), _p(raw), _st())
    ref = F.layer_norm(x, (256,), ga, be)
    tol = 1e-5 if prec == "fp32" else 2e-2
    assert (out.float().cpu() - ref).abs().max().item() <= tol
    assert (raw.float().cpu() - x.to(dt).float()).abs().max().item() == 0


@pytest.mark.parametrize("M,cus", [(1, 256), (77, 256), (1000, 256), (1000, 8), (5000, 16), (4700, 256)])
@pytest.mark.parametrize("oproj", [True, False])
def test_block_fused(M, cus, oproj):
    """Fused layer tail (k_block.hip): x' = x + O . Wo^T, x = x' + W2 . GELU(W1 . LN(x')), against the
    torch fp32 composition on the same bf16-rounded operands (O and the weights bf16; the LN output
    and the GELU output rounded to bf16 as the kernel does).  `cus` steers the rows per workgroup:
    a small CU count forces the 144-row tiles."""
    L = lib()
    D = 256
    g = torch.Generator().manual_seed(5 + M + cus)
    x = torch.randn(M, D, generator=g) * 2 + 0.3
    O = (torch.randn(M, D, generator=g)).to(torch.bfloat16)
    ga = 1 + 0.2 * torch.randn(D, generator=g)
    be = 0.1 * torch.randn(D, generator=g)
    Wo = (torch.randn(D, D, generator=g) / 16).to(torch.bfloat16)
    W1 = (torch.randn(3 * D, D, generator=g) / 16).to(torch.bfloat16)
    W2 = (torch.randn(D, 3 * D, generator=g) / 28).to(torch.bfloat16)
    dx = x.clone().cuda()
    dO, dWo = (O.cuda(), Wo.cuda()) if oproj else (None, None)
    d = [t.cuda() for t in (W1, W2, ga, be)]
    _run(L.lib().vap_test_block, _p(dx), _p(dO), M, _p(dWo), _p(d[0]), _p(d[1]), _p(d[2]), _p(d[3]), cus, _st())
    xp = x + O.float() @ Wo.float().t() if oproj else x
    a = F.layer_norm(xp, (D,), ga, be).to(torch.bfloat16).float()
    hdn = F.gelu(a @ W1.float().t()).to(torch.bfloat16).float()
    ref = xp + hdn @ W2.float().t()
    err = (dx.cpu() - ref).abs().max().item()
    assert err <= 2e-3 * max(1.0, ref.abs().max().item()), f"block M={M} cus={cus} oproj={oproj}: {err}"


@pytest.mark.parametrize("M", [1, 77, 1000, 4700])
@pytest.mark.parametrize("mode", ["oproj_qc", "qkv", "qkv_kvc"])
def test_lnproj_fused(M, mode):
    """Fused LayerNorm'd projections (k_block.hip lnproj): oproj_qc = x' = x + O . Wo^T (stored) and
    LN(x') . Wqc^T; qkv = LN(x) . Wqkv^T; qkv_kvc = that plus the raw-row cross K/V x . Wkv^T, against
    the torch fp32 composition on the same bf16-rounded operands (bf16 outputs)."""
    L = lib()
    D = 256
    g = torch.Generator().manual_seed(11 + M)
    x = torch.randn(M, D, generator=g) * 2 + 0.3
    O = torch.randn(M, D, generator=g).to(torch.bfloat16)
    ga = 1 + 0.2 * torch.randn(D, generator=g)
    be = 0.1 * torch.randn(D, generator=g)
    oproj = mode == "oproj_qc"
    np_, nr = (1, 0) if oproj else (3, 2 if mode == "qkv_kvc" else 0)
    Wo = (torch.randn(D, D, generator=g) / 16).to(torch.bfloat16)
    Wp = (torch.randn(np_ * D, D, generator=g) / 16).to(torch.bfloat16)
    Wr = (torch.randn(max(nr, 1) * D, D, generator=g) / 16).to(torch.bfloat16)
    dx = x.clone().cuda()
    cp = torch.zeros(M, np_ * D, dtype=torch.bfloat16, device="cuda")
    cr = torch.zeros(M, max(nr, 1) * D, dtype=torch.bfloat16, device="cuda")
    d = [t.cuda() for t in (O, Wo, Wp, Wr, ga, be)]
    _run(L.lib().vap_test_lnproj, _p(dx), _p(d[0]) if oproj else None, M, _p(d[1]) if oproj else None, _p(d[2]),
         np_, _p(d[3]) if nr else None, nr, _p(cp), _p(cr) if nr else None, _p(d[4]), _p(d[5]), _st())
    xp = x + O.float() @ Wo.float().t() if oproj else x
    assert (dx.cpu() - xp).abs().max().item() <= 1e-4 * max(1.0, xp.abs().max().item()), "x'"
    a = F.layer_norm(xp, (D,), ga, be).to(torch.bfloat16).float()
    ref = a @ Wp.float().t()
    err = (cp.float().cpu() - ref).abs().max().item()
    assert err <= 1e-2 * max(1.0, ref.abs().max().item()), f"cp {mode} M={M}: {err}"
    if nr:
        refr = x.to(torch.bfloat16).float() @ Wr.float().t()
        errr = (cr.float().cpu() - refr).abs().max().item()
        assert errr <= 1e-2 * max(1.0, refr.abs().max().item()), f"cr M={M}: {errr}"


@pytest.mark.parametrize("B,T", [(1, 37), (2, 1000), (3, 129)])
def test_heads_fused(B, T):
    """Fused combinator + vap_head (k_block.hip heads_kernel): logits = (GELU(LN(x1 Wa^T)) +
    GELU(LN(x2 Wb^T))) Wh^T + bh with one shared LayerNorm (modules.py:434-449, model.py:257-261),
    against the torch fp32 composition on the same bf16 operands (h rounded to bf16 as the kernel
    feeds it to the head GEMM; the kernel's GELU is the sigmoid fit, |error| <= 2.7e-4)."""
    L = lib()
    D = 256
    g = torch.Generator().manual_seed(31 + B * T)
    x = (torch.randn(2 * B, T, D, generator=g) * 1.5).to(torch.bfloat16)
    Wa, Wb, Wh = [(torch.randn(D, D, generator=g) / 16).to(torch.bfloat16) for _ in range(3)]
    ga = 1 + 0.2 * torch.randn(D, generator=g)
    be = 0.1 * torch.randn(D, generator=g)
    hb = 0.1 * torch.randn(D, generator=g)
    vw = 0.05 * torch.randn(D, generator=g)
    vb = 0.1 * torch.randn(1, generator=g)
    out = torch.full((B, T, D), 7.0, device="cuda")
    vad = torch.full((B, T, 2), 7.0, device="cuda")
    d = [t.cuda() for t in (x, Wa, Wb, Wh, ga, be, hb, vw, vb)]
    _run(L.lib().vap_test_heads, _p(d[0]), B, T, _p(d[1]), _p(d[2]), _p(d[3]), _p(d[4]), _p(d[5]), _p(d[6]), _p(d[7]),
         _p(d[8]), _p(out), _p(vad), _st())
    vref = (x.float().view(B, 2, T, D) @ vw + vb).permute(0, 2, 1)
    verr = (vad.cpu() - vref).abs().max().item()
    assert verr <= 1e-4 * max(1.0, vref.abs().max().item()), f"heads vad B={B} T={T}: {verr}"
    xf = x.float().view(B, 2, T, D)
    h = F.gelu(F.layer_norm(xf[:, 0] @ Wa.float().t(), (D,), ga, be)) + \
        F.gelu(F.layer_norm(xf[:, 1] @ Wb.float().t(), (D,), ga, be))
    ref = h.to(torch.bfloat16).float() @ Wh.float().t() + hb
    err = (out.cpu() - ref).abs().max().item()
    assert err <= 1e-2 * max(1.0, ref.abs().max().item()), f"heads B={B} T={T}: {err}"
