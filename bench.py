#!/usr/bin/env python3
"""Benchmark: VapGPT.probs (forward + probs epilogue) on batches of synthetic 20 s stereo clips.

Workload (BASELINE.json configs[1]): batch 64 x 20 s stereo @ 16 kHz per GPU, 50 Hz frames, bf16
perf mode (fp32 accumulate).  One "step" = model.probs(waveform) over the rank's batch, inputs
already resident in HBM.  With --gpus N > 1 (torchrun, one process per GPU, RCCL) every rank
processes its own 64 clips (clip seeds = global clip index: data-parallel shards, weak scaling)
and the compact per-frame outputs (p_now, p_future, vad, H) are gathered to rank 0 with one RCCL
gather per step (north_star: "single RCCL gather over xGMI for the output probabilities").

Prints ONE JSON line (rank 0) with the driver's contract fields plus `roofline` (dominant kernel,
HIP-event timed inside the timed region) and `cpu_baseline` (the CPU oracle on a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "audio-seconds/sec (whole node), 20s stereo @16kHz batch, 1/2/4/8 MI355X"
PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3}  # MI355X dense MFMA peaks (MI355X_MICROARCH.md)
CLASSES = ["conv0", "conv1", "conv234", "lstm_proj", "lstm_rec", "downsample", "tr_gemm", "attn", "norm", "heads"]


def class_flops(B: int, n: int, heads: int = 4, channel_layers: int = 1, cross_layers: int = 3, lstm_layers: int = 1):
    """Algorithmic FLOPs per step for each kernel class (2 per MAC; causal attention counts j <= i)."""
    from voiceactivityprojection_amd._native import frame_lengths

    L = frame_lengths(n)
    S, T, D = 2 * B, L[5], 256
    f = {}
    f["conv0"] = 2.0 * S * L[0] * D * 10
    f["conv1"] = 2.0 * S * L[1] * D * (D * 8)
    f["conv234"] = 2.0 * S * (L[2] + L[3] + L[4]) * D * (D * 4)
    f["lstm_proj"] = 2.0 * S * L[4] * 4 * D * D * lstm_layers
    f["lstm_rec"] = 2.0 * S * L[4] * 4 * D * D * lstm_layers
    f["downsample"] = 2.0 * S * T * D * (D * 5)
    per_layer_self = 2.0 * S * T * D * (3 * D + D + 3 * D + 3 * D)  # qkv, proj, ffn up, ffn down
    per_layer_cross = 2.0 * S * T * D * (2 * D + D + D)  # kv_c, q_c, proj_c
    f["tr_gemm"] = (channel_layers + cross_layers) * per_layer_self + cross_layers * per_layer_cross
    attn_one = 2.0 * 2 * heads * (T * (T + 1) / 2) * (D // heads)  # QK^T + PV, causal
    f["attn"] = S * attn_one * (channel_layers + 2 * cross_layers)
    f["norm"] = 0.0
    f["heads"] = 2.0 * B * T * D * (2 * D + 256) + 2.0 * S * T * D
    return f, L


def cpu_baseline(seconds: float, sd_np, budget_s: float = 12.0, max_clips: int = 32):
    """Time the CPU oracle (torch fp32 restatement of the reference) on a bounded sample."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import vap_oracle as O
    from voiceactivityprojection_amd.weights import synthetic_waveform

    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    sd = O.state_dict_to_torch(sd_np)
    n = int(seconds * 16000)
    O.probs(torch.from_numpy(synthetic_waveform(0, 16000 * 3)[None]), sd)  # warm-up
    done, t0 = 0, time.perf_counter()
    while done < max_clips:
        O.probs(torch.from_numpy(synthetic_waveform(done, n)[None]), sd)
        done += 1
        if time.perf_counter() - t0 > budget_s:
            break
    el = time.perf_counter() - t0
    return {"value": round(done * seconds / el, 3), "unit": "audio-s/s", "cores": threads, "kind": "port",
            "sample": f"{done} x {seconds:g} s stereo clip(s), batch 1, oracle/vap_oracle.py fp32 on "
                      f"{threads} host threads ({el:.1f} s)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64, help="clips per GPU")
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gather-probs", action="store_true", help="also gather the 256-way probs to rank 0")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as tdist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from vap.model import VapGPT
    from voiceactivityprojection_amd import _native as N
    from voiceactivityprojection_amd.weights import synthetic_batch, synthetic_state_dict

    sd_np = synthetic_state_dict(seed=0)
    model = VapGPT(precision=args.precision)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd_np.items()}, strict=True)
    model = model.to(dev).eval()

    B, n = args.batch, int(args.seconds * 16000)
    wav = torch.from_numpy(synthetic_batch(rank * B, B, n)).to(dev)
    flops, L = class_flops(B, n)
    if args.precision == "bf16":  # conv0 is fused into the conv1 kernel (k_conv01.hip)
        flops["conv1"] += flops["conv0"]
        flops["conv0"] = 0.0
    T = L[5]

    def step():
        out = model.probs(wav)
        if dist:
            keys = ["p_now", "p_future", "vad", "H"] + (["probs"] if args.gather_probs else [])
            for k in keys:
                t = out[k].contiguous()
                bufs = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
                tdist.gather(t, bufs, dst=0)
        return out

    # warm-up (includes weight packing)
    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize(dev)

    # per-class breakdown (one extra untimed step per class) to find the dominant kernel
    h = model._native(dev)
    lib = N.lib()
    breakdown = {}
    for cls in CLASSES:
        N.check(lib.vap_timing(h, N.KERNEL_CLASS[cls]))
        model.probs(wav)
        tot, cnt = __import__("ctypes").c_double(), __import__("ctypes").c_int()
        N.check(lib.vap_timing_read(h, __import__("ctypes").byref(tot), __import__("ctypes").byref(cnt)))
        breakdown[cls] = round(tot.value, 4)
    N.check(lib.vap_timing(h, 0))
    # the roofline is reported for the dominant kernel ON THE CRITICAL PATH (the caller's stream):
    # the LSTM recurrence runs as one persistent launch on a side stream, overlapped with (and
    # gated by) the front / back ends, so its launch time is mostly waiting, not work
    # (single-kernel classes only: tr_gemm / heads mix several kernels)
    dominant = max(("conv1", "conv234", "lstm_proj", "downsample", "attn"), key=breakdown.get)

    # timed region: K steps, HIP events around every launch of the dominant kernel class
    N.check(lib.vap_timing(h, N.KERNEL_CLASS[dominant]))
    if dist:
        tdist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        tdist.barrier()
    el = time.perf_counter() - t0
    import ctypes

    tot, cnt = ctypes.c_double(), ctypes.c_int()
    N.check(lib.vap_timing_read(h, ctypes.byref(tot), ctypes.byref(cnt)))
    N.check(lib.vap_timing(h, 0))
    if dist:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        el = float(t.item())

    if rank == 0:
        audio_s = world * B * args.seconds * args.steps
        value = audio_s / el
        dom_ms_per_launch = tot.value / max(1, cnt.value)
        launches_per_step = max(1, cnt.value // args.steps)
        flop_per_launch = flops[dominant] / launches_per_step
        achieved = flop_per_launch / (dom_ms_per_launch * 1e-3) / 1e12
        peak = PEAK_TFLOPS[args.precision]
        # HBM traffic of the dominant kernel: PMC-measured bytes per output row (profiles/, collected
        # by tools/pmc_traffic.sh on the serial schedule: PMC windows of overlapped kernels are polluted
        # by the concurrent LSTM) x the rows of one launch here
        traffic, traffic_src = None, None
        tp = os.path.join(REPO, "profiles", "r2_traffic_pmc.json")  # the current conv01 kernel (v11)
        if dominant == "conv1" and args.precision == "bf16" and os.path.exists(tp):
            per_row = json.load(open(tp))["conv1"]["hbm_bytes_per_row"]
            rows_per_launch = 2 * B * L[1] / launches_per_step
            traffic = round(per_row * rows_per_launch / 1e9, 3)
            traffic_src = "profiles/r2_traffic_pmc.json (GB per launch)"
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "audio-s/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.precision, "data": "synthetic",
            "config": {"workload": f"batch={B} x {args.seconds:g}s stereo @16kHz per GPU, 50Hz frames (T={T}), "
                                   f"{args.precision} (BASELINE.json configs[1])",
                       "global_batch": world * B, "seconds_per_clip": args.seconds, "frames": T,
                       "parallelism": f"dp{world}", "step": "VapGPT.probs (forward + probs epilogue + labels/loss)"
                                                            + (" + RCCL gather to rank 0" if dist else "")},
            "roofline": {"kernel": dominant, "bound": "mfma", "achieved": round(achieved, 2), "peak": peak,
                         "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "flop_per_launch": flop_per_launch, "ms_per_launch": round(dom_ms_per_launch, 4),
                         "launches": cnt.value},
            "breakdown_ms_per_step": breakdown,
            "breakdown_note": "ms of each kernel class per step (HIP events on its stream); lstm_rec is one persistent "
                              "side-stream launch overlapped with the caller-stream classes (its time includes "
                              "waiting for the time chunks), the other classes run back to back on the caller's stream",
            "model_tflops_per_s": round(sum(flops.values()) * args.steps * world / el / 1e12, 2),
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.seconds, sd_np)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
