#!/usr/bin/env python3
"""Kernel microbenchmarks through the test ABI (GPU box): isolated per-launch times of the
transformer row kernels, the attention and the generic GEMM at the bench's shapes.

    python tools/mb_kernels.py [--which rows,attn,gemm] [--rows 81920] [--iters 50]
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


def bench_rows(lib, dev, st, iters, M):
    """The transformer row kernels (k_block.hip) at one layer-chunk of M rows: LN + QKV + raw cross
    K/V, out-projection + LN + cross Q, LN + QKV, and the fused layer tail (out-proj + LN + FFN)."""
    g = torch.Generator(device="cpu").manual_seed(3)
    D = 256
    x = torch.randn(M, D, generator=g).to(dev)
    ga = (1 + 0.1 * torch.randn(D, generator=g)).to(dev)
    be = (0.1 * torch.randn(D, generator=g)).to(dev)

    def packed(n, k, scale):
        W = (torch.randn(n, k, generator=g) * scale).to(torch.bfloat16).to(dev)
        Wp = torch.empty_like(W)
        _native.check(lib.vap_test_pack_weight(ptr(W), ptr(Wp), n, k, st))
        return Wp
    W1p, W2p, Wop = packed(3 * D, D, 1 / 16), packed(D, 3 * D, 1 / 28), packed(D, D, 1 / 16)
    Wqkv, Wkv, Wq = packed(3 * D, D, 1 / 16), packed(2 * D, D, 1 / 16), packed(D, D, 1 / 16)
    O = torch.randn(M, D, generator=g).to(torch.bfloat16).to(dev)
    cp = torch.empty(M, 3 * D, device=dev, dtype=torch.bfloat16)
    cr = torch.empty(M, 2 * D, device=dev, dtype=torch.bfloat16)
    cus = int(os.environ.get("MB_CUS", "0"))

    def block():
        _native.check(lib.vap_test_block_packed(ptr(x), ptr(O), M, ptr(Wop), ptr(W1p), ptr(W2p), ptr(ga), ptr(be),
                                                cus, st))

    def qkv_kv():
        _native.check(lib.vap_test_lnproj_packed(ptr(x), None, M, None, ptr(Wqkv), 3, ptr(Wkv), 2, ptr(cp), ptr(cr),
                                                 ptr(ga), ptr(be), st))

    def qkv():
        _native.check(lib.vap_test_lnproj_packed(ptr(x), None, M, None, ptr(Wqkv), 3, None, 0, ptr(cp), None,
                                                 ptr(ga), ptr(be), st))

    def oproj_q():
        _native.check(lib.vap_test_lnproj_packed(ptr(x), ptr(O), M, ptr(Wop), ptr(Wq), 1, None, 0, ptr(cp), None,
                                                 ptr(ga), ptr(be), st))
    res = {}
    for name, fn, n_mac in [("block", block, D * D + 2 * 3 * D * D), ("lnproj_qkv_kv", qkv_kv, 5 * D * D),
                            ("lnproj_qkv", qkv, 3 * D * D), ("lnproj_oproj_q", oproj_q, 2 * D * D)]:
        us = timeit(fn, iters)
        res[name] = dict(us=round(us, 2), tflops=round(2.0 * M * n_mac / us / 1e6, 1))
        print(name, res[name], flush=True)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=81920, help="rows of the row-kernel launches")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--which", default="rows,attn")
    ap.add_argument("--case", default="", help="only GEMM cases whose name contains this")
    ap.add_argument("--attn-seqs", type=int, default=128, help="sequences of the attention benchmark")
    ap.add_argument("--attn-frames", type=int, default=1000)
    args = ap.parse_args()
    lib = _native.lib()
    dev = torch.device("cuda:0")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = {}
    if "attn" in args.which:
        res.update(bench_attn(lib, dev, st, args.iters, S=args.attn_seqs, T=args.attn_frames))
    if "rows" in args.which:
        res.update(bench_rows(lib, dev, st, args.iters, args.rows))
    if "gemm" in args.which:
        res.update(bench_gemm(lib, dev, st, args.iters, args.case))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
