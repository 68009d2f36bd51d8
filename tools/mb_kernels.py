#!/usr/bin/env python3
"""Kernel microbenchmarks through the test ABI (GPU box): isolated per-launch times of the
transformer projection kernels at the bench's per-range shape (32 sequences x 1000 frames).

    python tools/mb_kernels.py [--rows 32000] [--iters 50]
"""
import argparse
import ctypes
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from voiceactivityprojection_amd import _native  # noqa: E402


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def timeit(fn, iters):
    st = torch.cuda.current_stream()
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(iters):
        fn()
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters  # us


def bench_attn(lib, dev, st, iters, S=32, T=1000, H=4):
    """Causal AliBi attention at the engine's layout: Q/K/V columns of one [S][T][768] bf16 buffer."""
    g = torch.Generator(device="cpu").manual_seed(1)
    qkv = (torch.randn(S, T, 768, generator=g) * 2).to(torch.bfloat16).to(dev)
    O = torch.empty(S, T, 256, device=dev, dtype=torch.bfloat16)
    slopes = torch.tensor([0.25, 0.0625, 0.015625, 0.00390625], device=dev)
    scale = 1.0 / 16
    res = {}
    for kv_swap in (0, 1):
        def run():
            _native.check(lib.vap_test_attention(1, ctypes.c_void_p(qkv.data_ptr()), 768, T * 768,
                                                 ctypes.c_void_p(qkv.data_ptr() + 512), 768, T * 768,
                                                 ctypes.c_void_p(qkv.data_ptr() + 1024), 768, T * 768,
                                                 ptr(O), 256, T * 256, ptr(slopes), S, T, H, kv_swap,
                                                 ctypes.c_float(scale), st))
        us = timeit(run, iters)
        # reference on 4 sequences (fp32 math on the bf16 inputs)
        q = qkv[:4, :, :256].float().view(4, T, H, 64).transpose(1, 2)
        src = qkv[[1, 0, 3, 2]] if kv_swap else qkv[:4]
        k = src[:, :, 256:512].float().view(4, T, H, 64).transpose(1, 2)
        v = src[:, :, 512:].float().view(4, T, H, 64).transpose(1, 2)
        i = torch.arange(T, device=dev)
        bias = slopes.view(H, 1, 1) * (i.view(1, 1, T) - i.view(1, T, 1)).float()
        bias = bias.masked_fill(i.view(1, 1, T) > i.view(1, T, 1), float("-inf"))
        att = torch.softmax(q @ k.transpose(-1, -2) * scale + bias, -1) @ v
        ref = att.transpose(1, 2).reshape(4, T, 256)
        err = (O[:4].float() - ref).abs().max().item()
        flops = S * H * (T * (T + 1) / 2) * 64 * 4
        res[f"attn_kv{kv_swap}"] = dict(us=round(us, 2), tflops=round(flops / us / 1e6, 1), max_err=round(err, 4))
        print(f"attn_kv{kv_swap}", res[f"attn_kv{kv_swap}"], flush=True)
    return res


def bench_gemm(lib, dev, st, iters, only=""):
    """Generic implicit-conv GEMM (bf16) at the front-end / FFN shapes of one range (32 sequences)."""
    g = torch.Generator(device="cpu").manual_seed(2)
    res = {}
    D = 256
    gamma = (1 + 0.1 * torch.randn(D, generator=g)).to(dev)
    beta = (0.1 * torch.randn(D, generator=g)).to(dev)
    bias = (0.1 * torch.randn(4 * D, generator=g)).to(dev)
    # (name, rows_in_per_seq, lda, K, N, M_per_seq, norm, act, out_f32, residual)
    cases = [("conv2_cn_relu", 16002, 512, 1024, 256, 8000, 1, 1, 0, 0),
             ("conv2_plain", 16002, 512, 1024, 256, 8000, 0, 0, 0, 0),
             ("conv3_cn_relu", 8002, 512, 1024, 256, 4000, 1, 1, 0, 0),
             ("lstm_proj", 2000, 256, 256, 1024, 2000, 0, 0, 0, 0),
             ("ff2_resid", 1000, 768, 768, 256, 1000, 0, 0, 1, 1),
             ("ksweep_k512", 16002, 512, 512, 256, 8000, 0, 0, 0, 0),
             ("ksweep_k2048", 16002, 512, 2048, 256, 8000, 0, 0, 0, 0),
             ("ksweep_k4096", 16002, 512, 4096, 256, 8000, 0, 0, 0, 0)]
    S = 32
    for name, rin, lda, K, N, M, norm, act, out_f32, resid in cases:
        if only and only not in name:
            continue
        A = (torch.randn(S, rin, lda if lda > D else D, generator=g) * 0.5).to(torch.bfloat16).to(dev)
        a_seq = A.shape[1] * A.shape[2]
        W = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(torch.bfloat16).to(dev)
        C = torch.empty(S, M, N, device=dev, dtype=torch.float32 if out_f32 else torch.bfloat16)
        add = torch.randn(S, M, N, generator=g).to(dev) if resid else None

        def run():
            _native.check(lib.vap_test_gemm(1, ptr(A), lda, a_seq, ptr(W), K, N, ptr(bias) if name == "lstm_proj" else None,
                                            M, S, ptr(C), N, M * N, ptr(add), N, M * N,
                                            ptr(gamma) if norm else None, ptr(beta) if norm else None,
                                            norm, act, out_f32, st))
        us = timeit(run, iters)
        flops = 2.0 * S * M * N * K
        res[name] = dict(us=round(us, 2), tflops=round(flops / us / 1e6, 1))
        print(name, res[name], flush=True)
    # reference point for the shape (timing only): hipBLASLt via torch.matmul, plain GEMM
    if not only or only == "ref":
        for name, M, K, N in [("ref_hipblaslt_256000x1024x256", 256000, 1024, 256),
                              ("ref_hipblaslt_64000x256x1024", 64000, 256, 1024),
                              ("ref_hipblaslt_8192x8192x8192", 8192, 8192, 8192)]:
            a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
            us = timeit(lambda: torch.matmul(a, w.t()), max(3, iters // 5))
            res[name] = dict(us=round(us, 2), tflops=round(2.0 * M * N * K / us / 1e6, 1))
            print(name, res[name], flush=True)
    return res


def bench_ffn(lib, dev, st, iters, M):
    """Fused FFN block vs the unfused row-panel up + GEMM down, at one layer-chunk (M rows)."""
    g = torch.Generator(device="cpu").manual_seed(3)
    D = 256
    x0 = torch.randn(M, D, generator=g).to(dev)
    x = x0.clone()
    ga = (1 + 0.1 * torch.randn(D, generator=g)).to(dev)
    be = (0.1 * torch.randn(D, generator=g)).to(dev)
    W1 = (torch.randn(3 * D, D, generator=g) / 16).to(torch.bfloat16).to(dev)
    W2 = (torch.randn(D, 3 * D, generator=g) / 28).to(torch.bfloat16).to(dev)
    FF = torch.empty(M, 3 * D, device=dev, dtype=torch.bfloat16)

    W1p, W2p = torch.empty_like(W1), torch.empty_like(W2)
    _native.check(lib.vap_test_pack_weight(ptr(W1), ptr(W1p), 3 * D, D, st))
    _native.check(lib.vap_test_pack_weight(ptr(W2), ptr(W2p), D, 3 * D, st))

    def fused():
        _native.check(lib.vap_test_ffn_packed(ptr(x), M, ptr(W1p), ptr(W2p), ptr(ga), ptr(be), st))

    def unfused():
        _native.check(lib.vap_test_rowpanel(ptr(x), D, M, ptr(W1), D, 3 * D, ptr(FF), 3 * D, None, ptr(ga), ptr(be),
                                            1, 1, st))
        _native.check(lib.vap_test_gemm(1, ptr(FF), 3 * D, M * 3 * D, ptr(W2), 3 * D, D, None, M, 1, ptr(x), D, M * D,
                                        ptr(x), D, M * D, None, None, 0, 0, 1, st))
    Wo = (torch.randn(D, D, generator=g) / 16).to(torch.bfloat16).to(dev)
    Wop = torch.empty_like(Wo)
    _native.check(lib.vap_test_pack_weight(ptr(Wo), ptr(Wop), D, D, st))
    O = torch.randn(M, D, generator=g).to(torch.bfloat16).to(dev)
    cus = int(os.environ.get("MB_CUS", "248"))

    def block():  # out-proj + residual + LN + FFN + residual in one launch
        _native.check(lib.vap_test_block_packed(ptr(x), ptr(O), M, ptr(Wop), ptr(W1p), ptr(W2p), ptr(ga), ptr(be),
                                                cus, st))

    def oproj_ffn():  # the pair it replaces: row-panel out-proj (+ residual) then the fused FFN
        _native.check(lib.vap_test_rowpanel(ptr(O), D, M, ptr(Wop), D, D, ptr(x), D, ptr(x), None, None, 16, 2, st))
        fused()

    res = {}
    for name, fn in [("ffn_fused", fused), ("ffn_unfused", unfused), ("oproj_ffn", oproj_ffn), ("block", block)]:
        us = timeit(fn, iters)
        res[name] = dict(us=round(us, 2), tflops=round(2.0 * M * 2 * 3 * D * D / us / 1e6, 1))
        print(name, res[name], flush=True)
    return res


def pack_rowpanel(W):
    """[N][256] bf16 -> the packed row-panel layout [N/256][8][16][64][8] (lane = (k%32)/8*16 + n%16)."""
    N = W.shape[0]
    return W.view(N // 256, 16, 16, 8, 4, 8).permute(0, 3, 1, 4, 2, 5).contiguous()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32000)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--which", default="rowpanel,attn")
    ap.add_argument("--case", default="", help="only GEMM cases whose name contains this")
    ap.add_argument("--packed", action="store_true", help="row-panel W in the packed layout")
    ap.add_argument("--attn-seqs", type=int, default=32, help="sequences of the attention benchmark")
    ap.add_argument("--attn-frames", type=int, default=1000)
    args = ap.parse_args()
    lib = _native.lib()
    dev = torch.device("cuda:0")
    M, D = args.rows, 256
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(M, D, generator=g).to(dev)
    xb = x.to(torch.bfloat16)
    gamma = (1 + 0.1 * torch.randn(D, generator=g)).to(dev)
    beta = (0.1 * torch.randn(D, generator=g)).to(dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = {}
    if "attn" in args.which:
        res.update(bench_attn(lib, dev, st, args.iters, S=args.attn_seqs, T=args.attn_frames))
    if "ffn" in args.which:
        res.update(bench_ffn(lib, dev, st, args.iters, args.rows))
    if "gemm" in args.which:
        res.update(bench_gemm(lib, dev, st, args.iters, args.case))
    if "rowpanel" not in args.which:
        print(json.dumps(res))
        return
    for name, amode, epi, N in [("qkv_ln", 1, 0, 768), ("q_ln", 1, 0, 256), ("ff1_ln_gelu", 1, 1, 768),
                                ("kv_raw", 2, 0, 512), ("proj_resid", 0, 2, 256)]:
        W = (torch.randn(N, D, generator=g) / 16).to(dev).to(torch.bfloat16)
        A = xb if amode == 0 else x
        add = torch.randn(M, N, generator=g).to(dev) if epi == 2 else None
        C = torch.empty(M, N, device=dev, dtype=torch.float32 if epi == 2 else torch.bfloat16)

        Wk = pack_rowpanel(W) if args.packed else W

        def run():
            _native.check(lib.vap_test_rowpanel(ptr(A), D, M, ptr(Wk), D, N, ptr(C), N, ptr(add),
                                                ptr(gamma) if amode == 1 else None,
                                                ptr(beta) if amode == 1 else None,
                                                amode | (16 if args.packed else 0), epi, st))
        us = timeit(run, args.iters)
        # check against torch (fp32 math on the bf16-rounded operands)
        a = x
        if amode == 1:
            a = torch.nn.functional.layer_norm(x, (D,), gamma, beta, 1e-5)
        a = a.to(torch.bfloat16).float()
        ref = a @ W.float().t()
        if epi == 1:
            ref = torch.nn.functional.gelu(ref)
        if epi == 2:
            ref = ref + add
        err = (C.float() - ref).abs().max().item()
        flops = 2.0 * M * N * D
        byts = M * D * (2 if amode == 0 else 4) + M * N * (4 if epi == 2 else 2) + (M * N * 4 if epi == 2 else 0)
        res[name] = dict(us=round(us, 2), tflops=round(flops / us / 1e6, 1), tbps=round(byts / us / 1e6, 2),
                         max_err=round(err, 4))
        print(name, res[name], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
