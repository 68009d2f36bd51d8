#!/usr/bin/env python3
"""Kernel microbenchmarks through the test ABI (GPU box): isolated per-launch times of the
transformer projection kernels at the bench's per-range shape (32 sequences x 1000 frames).

    python tools/mb_kernels.py [--rows 32000] [--iters 50]
"""
import argparse
import ctypes
import json
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32000)
    ap.add_argument("--iters", type=int, default=50)
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
    for name, amode, epi, N in [("qkv_ln", 1, 0, 768), ("q_ln", 1, 0, 256), ("ff1_ln_gelu", 1, 1, 768),
                                ("kv_raw", 2, 0, 512), ("proj_resid", 0, 2, 256)]:
        W = (torch.randn(N, D, generator=g) / 16).to(dev).to(torch.bfloat16)
        A = xb if amode == 0 else x
        add = torch.randn(M, N, generator=g).to(dev) if epi == 2 else None
        C = torch.empty(M, N, device=dev, dtype=torch.float32 if epi == 2 else torch.bfloat16)

        def run():
            _native.check(lib.vap_test_rowpanel(ptr(A), D, M, ptr(W), D, N, ptr(C), N, ptr(add),
                                                ptr(gamma) if amode == 1 else None,
                                                ptr(beta) if amode == 1 else None, amode, epi, st))
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
