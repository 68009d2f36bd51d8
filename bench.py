#!/usr/bin/env python3
"""Benchmark: VapGPT.probs (forward + probs epilogue) on batches of synthetic 20 s stereo clips.

Workload (BASELINE.json configs[1]): batch 64 x 20 s stereo @ 16 kHz per GPU, 50 Hz frames, bf16
perf mode (fp32 accumulate).  One "step" = model.probs(waveform) over the rank's batch, inputs
already resident in HBM.

Multi-GPU (BASELINE configs[2]): ``--gpus N`` runs one process per GPU.  Under
torchrun (WORLD_SIZE set) this process is one rank; without it, ``--gpus N > 1`` starts torchrun
with N ranks as a child process before anything touches the GPU and exits with its code.  Every
rank processes its own 64 clips (clip seeds = global clip index: data-parallel shards, weak
scaling) and writes its outputs into one packed buffer (distributed.PackedOutputs: probs, vad,
p_now, p_future, H, loss); each step ships that buffer to rank 0 with ONE RCCL gather, issued
asynchronously so it overlaps the next step's compute (double-buffered).

Prints ONE JSON line (rank 0) with the driver's contract fields plus `roofline` (dominant kernel,
HIP-event timed inside the timed region) and `cpu_baseline` (the CPU oracle on a bounded sample).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
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
    from voiceactivityprojection_amd.utils import frame_lengths

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


def host_cpu_share():
    """The host CPUs this process may use: min(affinity mask, cgroup cpu.max quota, OMP_NUM_THREADS when
    the environment sets it).  On the GPU pool ``nproc`` shows the whole 256-CPU host, which the
    node's GPU jobs share; the pool grants 16 CPUs per GPU and sets OMP_NUM_THREADS=16, asking jobs to
    keep it, so the CPU baseline runs on exactly that share."""
    nproc = os.cpu_count() or 1
    share, src = nproc, "os.cpu_count"
    try:
        aff = len(os.sched_getaffinity(0))
        if aff < share:
            share, src = aff, "sched_getaffinity"
    except (AttributeError, OSError):
        pass
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max" and int(per) > 0 and int(int(q) / int(per)) < share:
            share, src = max(1, int(int(q) / int(per))), "cgroup cpu.max"
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) < share:
        share, src = int(omp), "OMP_NUM_THREADS (the pool's per-GPU CPU share)"
    return share, nproc, src


def cpu_baseline(seconds: float, sd_np, budget_s: float = 12.0, max_clips: int = 32, batch: int = 4):
    """Time the CPU oracle (torch fp32 restatement of the reference) on a bounded sample: batches of
    `batch` clips of the workload's length (the GPU workload's shape, fewer clips per call) until the
    budget is spent, on every host CPU this process may use (host_cpu_share)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import vap_oracle as O
    from voiceactivityprojection_amd.weights import synthetic_waveform

    threads, nproc, share_src = host_cpu_share()
    torch.set_num_threads(threads)
    sd = O.state_dict_to_torch(sd_np)
    n = int(seconds * 16000)
    O.probs(torch.from_numpy(synthetic_waveform(0, 16000 * 3)[None]), sd)  # warm-up
    done, calls, t0 = 0, 0, time.perf_counter()
    while done < max_clips:
        w = np.stack([synthetic_waveform(done + i, n) for i in range(batch)])
        O.probs(torch.from_numpy(w), sd)
        done += batch
        calls += 1
        if time.perf_counter() - t0 > budget_s:
            break
    el = time.perf_counter() - t0
    return {"value": round(done * seconds / el, 3), "unit": "audio-s/s", "cores": threads, "kind": "port",
            "nproc": nproc, "cores_source": share_src,
            "sample": f"{calls} call(s) of {batch} x {seconds:g} s stereo clips, oracle/vap_oracle.py fp32 on "
                      f"{threads} host threads = this process's CPU share ({share_src}; {el:.1f} s; nproc {nproc})"}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64, help="clips per GPU")
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gather", default="all", choices=["all", "compact"],
                    help="outputs shipped to rank 0: all six probs() outputs, or p_now/p_future/vad/H")
    # CPU rehearsal of the launcher / gather path (tests/test_bench_launcher.py): gloo ranks on the host
    # with a stub step that writes rank-tagged outputs; no GPU, no engine
    # HIP events around every dominant-kernel launch of EVERY timed step cost ~7 % of the step (each event
    # pair splits the two front-end streams' overlap); the last timed step carries them by default
    ap.add_argument("--roofline-events", type=int, default=1,
                    help="timed steps (the last ones) whose dominant-kernel launches carry HIP events (-1: all)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the secondary configurations measured after the headline at N=1 (C4, parity mode)")
    ap.add_argument("--stub", action="store_true", help=argparse.SUPPRESS)
    # tests: rank 1 of the stub writes clips shifted by one (the exact gather check must catch it)
    ap.add_argument("--stub-wrong-offset", action="store_true", help=argparse.SUPPRESS)
    # tests: the handle never publishes the recurrence's ready flag of this time chunk (vap_test_drop_ready)
    ap.add_argument("--test-drop-ready", type=int, default=-1, help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(args, argv) -> int:
    """--gpus N > 1 without a torchrun environment: start torchrun with N ranks (one process per GPU)
    running this script, as a CHILD process (this process has not touched the GPU), and return its
    exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.run(cmd, env=env).returncode


class _StubModel:
    """--stub: writes rank-tagged outputs (value = global clip index + key offset) so rank 0 can
    verify the gathered layout exactly."""

    def __init__(self, first_clip: int):
        self.first_clip = first_clip

    def probs(self, wav, out):
        for j, (k, v) in enumerate(out.items()):
            idx = torch.arange(v.shape[0], dtype=torch.float32).view(-1, *([1] * (v.dim() - 1)))
            v.copy_((self.first_clip + idx + 1000.0 * j).expand_as(v))
        return out

    def synchronize(self):
        pass


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch(args, argv)
    return run_rank(args)


def run_rank(args) -> int:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU is required")
    dist = world > 1
    import torch.distributed as tdist

    from voiceactivityprojection_amd.distributed import PackedOutputs, gather_packed
    from voiceactivityprojection_amd.utils import frame_lengths
    from voiceactivityprojection_amd.weights import synthetic_batch

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if args.stub:
        dev = torch.device("cpu")
        if dist:
            tdist.init_process_group("gloo")
    else:
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
        if dist:
            tdist.init_process_group("nccl", device_id=dev)

    B, n = args.batch, int(args.seconds * 16000)
    T = frame_lengths(n)[5]
    keys = ("probs", "vad", "p_now", "p_future", "H", "loss") if args.gather == "all" else ("p_now", "p_future", "vad", "H")
    if args.stub:
        model, wav, sd_np = _StubModel(rank * B + (1 if args.stub_wrong_offset and rank == 1 else 0)), None, None
    else:
        from vap.model import VapGPT
        from voiceactivityprojection_amd.weights import synthetic_state_dict

        sd_np = synthetic_state_dict(seed=0)
        model = VapGPT(precision=args.precision)
        model.load_state_dict({k: torch.from_numpy(v) for k, v in sd_np.items()}, strict=True)
        model = model.to(dev).eval()
        wav = torch.from_numpy(synthetic_batch(rank * B, B, n)).to(dev)
        if args.test_drop_ready >= 0:
            from voiceactivityprojection_amd import _native as N0

            N0.check(N0.lib().vap_test_drop_ready(model._native(dev), args.test_drop_ready))

    # double-buffered packed outputs: step i writes packs[i % 2] while the gather of step i - 1 runs
    packs = [PackedOutputs(B, T, dev, keys) for _ in range(2)]
    recvs = [[torch.empty_like(p.flat) for _ in range(world)] if dist and rank == 0 else None for p in packs]
    works = [None, None]
    state = {"i": 0}

    def step():
        j = state["i"] % 2
        state["i"] += 1
        if works[j] is not None:
            works[j].wait()  # the gather that last read this buffer (stream-ordered on RCCL)
        model.probs(wav, out=packs[j].views())
        if dist:
            works[j], _ = gather_packed(packs[j], dst=0, recv=recvs[j], async_op=True)

    def drain():
        for j in range(2):
            if works[j] is not None:
                works[j].wait()
                works[j] = None

    def device_sync():
        if not args.stub:
            torch.cuda.synchronize(dev)

    for _ in range(max(1, args.warmup)):  # warm-up (includes weight packing)
        step()
    drain()
    device_sync()
    model.synchronize()

    breakdown, dominant, lib, h, N = {}, None, None, None, None
    flops, L = class_flops(B, n)
    if args.precision == "bf16":  # conv0 is fused into the conv1 kernel (k_conv01.hip)
        flops["conv1"] += flops["conv0"]
        flops["conv0"] = 0.0
    if not args.stub:
        # per-class breakdown (one extra untimed forward per class) to find the dominant kernel
        from voiceactivityprojection_amd import _native as N

        h = model._native(dev)
        lib = N.lib()
        for cls in CLASSES:
            N.check(lib.vap_timing(h, N.KERNEL_CLASS[cls]))
            model.probs(wav, out=packs[0].views())
            tot, cnt = ctypes.c_double(), ctypes.c_int()
            N.check(lib.vap_timing_read(h, ctypes.byref(tot), ctypes.byref(cnt)))
            breakdown[cls] = round(tot.value, 4)
        N.check(lib.vap_timing(h, 0))
        model.synchronize()
        # the roofline is reported for the dominant kernel ON THE CRITICAL PATH (the caller's stream):
        # the LSTM recurrence runs as one persistent launch on a side stream, overlapped with (and
        # gated by) the front / back ends, so its launch time is mostly waiting, not work
        # (single-kernel classes only: tr_gemm / heads mix several kernels)
        dominant = max(("conv1", "conv234", "lstm_proj", "downsample", "attn"), key=breakdown.get)
        # the same class with the front end on ONE stream (one untimed forward): the kernel's own
        # duration, not shared with conv2..4 of the previous piece on the second front-end stream
        N.check(lib.vap_timing(h, -N.KERNEL_CLASS[dominant]))
        model.probs(wav, out=packs[0].views())
        iso_tot, iso_cnt = ctypes.c_double(), ctypes.c_int()
        N.check(lib.vap_timing_read(h, ctypes.byref(iso_tot), ctypes.byref(iso_cnt)))
        model.synchronize()
    ev_from = 0 if args.roofline_events < 0 else max(0, args.steps - args.roofline_events)
    if not args.stub and ev_from > 0:
        N.check(lib.vap_timing(h, 0))  # events only from step ev_from on

    # timed region: K steps (+ their gathers), HIP events around every launch of the dominant class
    if dist:
        tdist.barrier()
    device_sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if not args.stub and ev_from > 0 and i == ev_from:
            N.check(lib.vap_timing(h, N.KERNEL_CLASS[dominant]))
        step()
    drain()
    device_sync()
    model.synchronize()  # a timed-out recurrence hand-off fails the bench instead of reporting a number
    if dist:
        tdist.barrier()
    el = time.perf_counter() - t0

    tot, cnt = ctypes.c_double(), ctypes.c_int()
    if not args.stub:
        N.check(lib.vap_timing_read(h, ctypes.byref(tot), ctypes.byref(cnt)))
        N.check(lib.vap_timing(h, 0))
    if dist:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        el = float(t.item())

    gather_info = None
    if dist:
        last = (state["i"] - 1) % 2
        verified, checked = None, []
        if rank == 0:
            got = recvs[last]
            verified = bool(torch.equal(got[0], packs[last].flat))  # rank 0's own shard, bit for bit
            verified = verified and all(bool(torch.isfinite(g).all()) for g in got)
            # every rank's first and last clip recomputed here, ALONE (clip seed = global clip index), and
            # compared bit for bit with that rank's gathered region: batch invariance (every kernel is per
            # sequence) makes a one-clip run exact, so a rank that computed the wrong clips fails here
            one = PackedOutputs(1, T, dev, keys)
            for r in range(world):
                view = packs[last].views(B, flat=got[r])
                for i in sorted({0, B - 1}):
                    c = r * B + i
                    if args.stub:
                        _StubModel(c).probs(None, one.views())
                    else:
                        model.probs(torch.from_numpy(synthetic_batch(c, 1, n)).to(dev), out=one.views())
                    ok = all(torch.equal(view[k][i:i + 1], one.views()[k]) for k in keys)
                    checked.append({"rank": r, "clip": c, "bit_identical": ok})
                    verified = verified and ok
            if not args.stub:
                model.synchronize()
        gather_info = {"collective": "torch.distributed.gather" + (" (gloo)" if args.stub else " (RCCL)"),
                       "calls_per_step": 1, "bytes_per_rank": packs[0].flat.numel() * 4, "keys": list(keys),
                       "overlapped_with_next_step": True, "verified": verified,
                       "verification": "rank 0's shard bit for bit; every rank's first and last clip recomputed "
                                       "alone on rank 0 and compared bit for bit (batch invariance)",
                       "clips_checked": checked}

    if rank == 0:
        audio_s = world * B * args.seconds * args.steps
        value = audio_s / el
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "audio-s/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.precision, "data": "synthetic",
            "config": {"workload": f"batch={B} x {args.seconds:g}s stereo @16kHz per GPU, 50Hz frames (T={T}), "
                                   f"{args.precision} (BASELINE.json configs[{1 if world == 1 else 2}])",
                       "global_batch": world * B, "seconds_per_clip": args.seconds, "frames": T,
                       "parallelism": f"dp{world}", "step": "VapGPT.probs (forward + probs epilogue + labels/loss)"
                                                            + (" + one RCCL gather to rank 0" if dist else "")},
        }
        if gather_info is not None:
            line["gather"] = gather_info
        if not args.stub:
            ev_steps = args.steps - ev_from  # timed steps whose dominant launches carried events
            if cnt.value == 0:  # --roofline-events 0: the isolated pass's launches stand in
                tot, cnt, ev_steps = iso_tot, iso_cnt, 1
            dom_ms_per_launch = tot.value / max(1, cnt.value)
            launches_per_step = max(1, cnt.value // max(1, ev_steps))
            flop_per_launch = flops[dominant] / launches_per_step
            achieved = flop_per_launch / (dom_ms_per_launch * 1e-3) / 1e12
            peak = PEAK_TFLOPS[args.precision]
            # HBM traffic of the dominant kernel: PMC-measured bytes per output row (profiles/, collected
            # by tools/pmc_traffic.sh on the serial schedule: PMC windows of overlapped kernels are polluted
            # by the concurrent LSTM) x the rows of one launch here
            traffic, traffic_src = None, None
            tp = os.path.join(REPO, "profiles", "r4", "traffic_pmc_s6.json")  # the current conv01 kernel (round 4, session 6)
            if dominant == "conv1" and args.precision == "bf16" and os.path.exists(tp):
                per_row = json.load(open(tp))["conv1"]["hbm_bytes_per_row"]
                rows_per_launch = 2 * B * L[1] / launches_per_step
                traffic = round(per_row * rows_per_launch / 1e9, 3)
                traffic_src = "profiles/r4/traffic_pmc_s6.json (GB per launch)"
            line["roofline"] = {"kernel": dominant, "bound": "mfma", "achieved": round(achieved, 2), "peak": peak,
                                "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": traffic,
                                "traffic_source": traffic_src, "flop_per_launch": flop_per_launch,
                                "ms_per_launch": round(dom_ms_per_launch, 4), "launches": cnt.value,
                                "event_steps": ev_steps}
            if dominant in ("conv1", "conv234", "lstm_proj"):
                iso_ms = iso_tot.value / max(1, iso_cnt.value)
                iso_ach = flop_per_launch / (iso_ms * 1e-3) / 1e12
                line["roofline"]["concurrency"] = (
                    "timed region: the front end runs on two streams, so each launch shares the CUs with conv2..4 "
                    "and the gate projection of the previous piece (ms_per_launch is that shared duration); "
                    "isolated: the same launches with the front end on one stream (one untimed forward)")
                line["roofline"]["isolated"] = {"ms_per_launch": round(iso_ms, 4), "achieved": round(iso_ach, 2),
                                                "frac": round(iso_ach / peak, 4)}
            line["breakdown_ms_per_step"] = breakdown
            line["breakdown_note"] = ("ms of each kernel class per step (HIP events on its stream); lstm_rec is one "
                                      "persistent side-stream launch overlapped with the caller-stream classes (its "
                                      "time includes waiting for the time chunks); the front end runs on two "
                                      "streams (conv01 of piece k+1 beside conv2..4 + gate projection of piece k), "
                                      "the back end in two clip halves on two streams; a back-end class is timed in "
                                      "a forward with the back end on one stream")
            line["model_tflops_per_s"] = round(sum(flops.values()) * args.steps * world / el / 1e12, 2)
        if world == 1 and not args.stub:
            # the headline outputs of the last timed step against the reference's own outputs for clips
            # 0..3 of this batch (tests/golden/bench4_20s.npz), at the mode's stated tolerance
            fx = fixture_errors(packs[(state["i"] - 1) % 2].views(), B, args.seconds, args.precision)
            if fx is not None:
                line["parity"] = fx
            if not args.no_extras:
                line["extras"] = extras(args, model, dev, sd_np)
        if world == 1 and not args.no_cpu_baseline and not args.stub:
            line["cpu_baseline"] = cpu_baseline(args.seconds, sd_np)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    if dist:
        tdist.destroy_process_group()
    if gather_info is not None and rank == 0 and gather_info["verified"] is not True:
        print("bench.py: the gathered outputs failed the exact per-rank check", file=sys.stderr)
        return 3
    return 0


def fixture_errors(out, B: int, seconds: float, precision: str):
    """Max abs error of clips 0..3 of a bench batch (synthetic_batch(0, ...), 20 s) against the reference's
    outputs for the same clips (tests/golden/bench4_20s.npz, tools/gen_golden.py), per output, with the
    mode's stated tolerance (voiceactivityprojection_amd/tolerances.py)."""
    from voiceactivityprojection_amd.tolerances import TOL

    path = os.path.join(REPO, "tests", "golden", "bench4_20s.npz")
    if seconds != 20.0 or B < 4 or not os.path.exists(path):
        return None
    g = dict(np.load(path, allow_pickle=False))
    tol = TOL[precision]
    err = {}
    for k in ("vad", "p_now", "p_future", "H", "loss"):
        if k in out and k in g:
            err[k] = float(np.abs(out[k][:4].float().cpu().numpy() - g[k]).max())
    if "probs" in out and "probs_stride10" in g:
        err["probs"] = float(np.abs(out["probs"][:4, ::10].float().cpu().numpy() - g["probs_stride10"]).max())
    return {"reference_fixture": "tests/golden/bench4_20s.npz (clips 0..3 of this batch, reference outputs)",
            "max_abs_err": {k: float(f"{v:.3g}") for k, v in err.items()}, "tolerance": {k: tol[k] for k in err},
            "within_tolerance": all(err[k] <= tol[k] for k in err)}


def _leg(model, wav, steps: int, warmup: int, keys=None):
    """Steps of model.probs on a resident batch: (ms per step, outputs of the last step).  Like the
    headline loop, every step writes into the same preallocated outputs (the first warm-up step's)."""
    out = model.probs(wav)
    for _ in range(warmup - 1):
        model.probs(wav, out=out)
    torch.cuda.synchronize()
    model.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        model.probs(wav, out=out)
    torch.cuda.synchronize()
    model.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3, out


def extras(args, model, dev, sd_np, steps: int = 5, warmup: int = 3):
    """Secondary BASELINE configurations measured in the same run after the headline (N = 1, untimed by
    the headline): C4 (32 x 60 s, T = 3000, the headline's precision) and the fp32 parity mode on the
    headline workload (64 x 20 s) with its errors against the reference fixture."""
    from vap.model import VapGPT
    from voiceactivityprojection_amd.weights import synthetic_batch

    res = {}
    n4, B4 = 60 * 16000, 32
    wav4 = torch.from_numpy(synthetic_batch(0, B4, n4)).to(dev)
    ms, _ = _leg(model, wav4, steps, warmup)
    res["c4"] = {"value": round(B4 * 60.0 / (ms * 1e-3), 2), "unit": "audio-s/s", "ms_per_step": round(ms, 3),
                 "steps": steps, "warmup": warmup, "dtype": args.precision,
                 "config": "BASELINE.json configs[3]: batch=32 x 60s stereo @16kHz (T=3000, AliBi extrapolation), "
                           "1 GPU, VapGPT.probs"}
    del wav4
    if args.precision != "fp32":
        # the headline model's native handle goes first: its side streams would otherwise share the
        # process's GPU_MAX_HW_QUEUES (4) hardware queues with the fp32 model's, and a persistent
        # recurrence queued on the caller stream's hardware queue serialises the leg (measured 14 %
        # slower than the same mode alone: 43.8k vs 49.9k audio-s/s, profiles/r4/bench_s9.json)
        model._free_handle()
        torch.cuda.synchronize()
        B, n = args.batch, int(args.seconds * 16000)
        m32 = VapGPT(precision="fp32")
        m32.load_state_dict({k: torch.from_numpy(v) for k, v in sd_np.items()}, strict=True)
        m32 = m32.to(dev).eval()
        wav = torch.from_numpy(synthetic_batch(0, B, n)).to(dev)
        ms, out = _leg(m32, wav, steps, warmup)
        res["parity_mode"] = {"value": round(B * args.seconds / (ms * 1e-3), 2), "unit": "audio-s/s",
                              "ms_per_step": round(ms, 3), "steps": steps, "warmup": warmup, "dtype": "fp32",
                              "config": f"the headline workload (batch={B} x {args.seconds:g}s) in the fp32 parity mode",
                              "parity": fixture_errors(out, B, args.seconds, "fp32")}
        del m32, wav, out
    torch.cuda.empty_cache()
    return res


if __name__ == "__main__":
    sys.exit(main())
