#!/usr/bin/env python3
"""Streaming throughput (SURVEY config C5): rolling 10 s windows advanced by a 1 s hop; one push =
one step.  Metric: NEW audio-seconds per second over the whole node (streams x hop per step), as C5
counts it.  Reference loop: sds/run_sds.py:206-241 (roll the block into the window, probs() on the
whole window), run.py:23-92 step_extraction (keep the last step's frames).

    python tools/bench_stream.py [--gpus N] [--streams-per-gpu 16] [--steps 10] [--warmup 11]

Multi-GPU (BASELINE configs[4]: 128 streams over 8 GPUs): one process per GPU, exactly as bench.py --
under torchrun (WORLD_SIZE set) this process is one rank; without it, ``--gpus N > 1`` starts
torchrun with N ranks as a child process before anything touches the GPU.  Streams shard by rank:
rank r owns global streams [r*S, (r+1)*S) (S = --streams-per-gpu; the audio of stream g is the seeded
generator's clip 5000 + g), so the streams are independent and no collective sits on the data path.
Each push's new-hop outputs (probs, vad, p_now, p_future, H of the last 50 frames) are packed into one
buffer and shipped to rank 0 with ONE gather, issued asynchronously on a double-buffered pack so it
overlaps the next push.  After the timed loop rank 0 checks every rank's first and last stream of the
last push bit for bit against a full forward of that stream's final window (streaming outputs equal
the forward of the rolled window: tests/test_gpu_stream.py).

VAP_STREAM_REUSE=0 disables the CPC conv-row carry-over (full recompute per push) for an A/B;
VAP_STREAM_GRAPH=0 issues every push eagerly instead of replaying its captured hipGraph.
Inputs: the seeded synthetic waveform generator (no dataset), bf16, weights random-init.
``--stub`` rehearses the launcher and the gather on CPU ranks (gloo) with rank-tagged outputs.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

KEYS = ("probs", "vad", "p_now", "p_future", "H")
HOP, SR, WINDOW_S = 16000, 16000, 10.0


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--streams-per-gpu", "--streams", dest="streams", type=int, default=128,
                    help="streams per GPU (C5: 16 per GPU x 8; also reported at 128 per GPU)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=11, help="pushes before timing (10 fill the window)")
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--check-each", action="store_true",
                    help="push(check=True): wait for every push and check its hand-off (the real-time loop's "
                         "default); otherwise pushes are pipelined and checked once after the timed loop")
    ap.add_argument("--stub", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--stub-wrong-offset", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(args, argv) -> int:
    """--gpus N > 1 without torchrun: N ranks as a child process (this process has not touched the GPU)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.run(cmd, env=env).returncode


class _StubStream:
    """--stub: push() returns hop outputs tagged with (global stream, push index, key)."""

    def __init__(self, first: int, batch: int, hop_frames: int = 50):
        self.first, self.batch, self.hop_frames, self.pushes = first, batch, hop_frames, 0
        self.frames, self.reused_rows = 500, 0

    @staticmethod
    def expect(g: int, push: int, hop_frames: int = 50):
        shapes = {"probs": (hop_frames, 256), "vad": (hop_frames, 2), "p_now": (hop_frames, 2),
                  "p_future": (hop_frames, 2), "H": (hop_frames,)}
        return {k: torch.full(s, float(g + 1000 * push + 1e6 * j)) for j, (k, s) in enumerate(shapes.items())}

    def push(self, audio, check=True):
        self.pushes += 1
        per = [self.expect(self.first + b, self.pushes, self.hop_frames) for b in range(self.batch)]
        return {k: torch.stack([p[k] for p in per]) for k in KEYS}

    def synchronize(self):
        pass

    def graph_info(self):
        return None


def stream_audio(g: int, n: int) -> np.ndarray:
    from voiceactivityprojection_amd.weights import synthetic_waveform

    return synthetic_waveform(5000 + g, n)


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
        raise SystemExit(f"bench_stream.py: --gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU is required")
    dist = world > 1
    import torch.distributed as tdist

    from voiceactivityprojection_amd.distributed import PackedOutputs, gather_packed

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

    S = args.streams
    g0 = rank * S  # this rank's global streams [g0, g0 + S)
    n = HOP * (args.warmup + args.steps)
    if args.stub:
        m = None
        st = _StubStream(g0 + (1 if args.stub_wrong_offset and rank == 1 else 0), S)
        audio = torch.zeros(S, 2, n)
    else:
        from vap.model import VapGPT
        from voiceactivityprojection_amd.weights import synthetic_state_dict

        m = VapGPT(precision=args.precision)
        m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0).items()}, strict=True)
        m = m.to(dev).eval()
        st = m.stream(S, context_time=WINDOW_S, hop_time=HOP / SR)
        audio = torch.from_numpy(np.stack([stream_audio(g0 + b, n) for b in range(S)])).to(dev)
    F = st.hop_frames if not args.stub else 50

    # double-buffered packed hop outputs: push i writes packs[i % 2] while the gather of push i - 1 runs
    packs = [PackedOutputs(S, F, dev, KEYS) for _ in range(2)]
    recvs = [[torch.empty_like(p.flat) for _ in range(world)] if dist and rank == 0 else None for p in packs]
    works = [None, None]
    state = {"i": 0}

    def step(k):
        j = state["i"] % 2
        state["i"] += 1
        if works[j] is not None:
            works[j].wait()
        out = st.push(audio[..., k * HOP:(k + 1) * HOP], check=args.check_each)
        v = packs[j].views()
        for key in KEYS:
            v[key].copy_(out[key])
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

    for k in range(args.warmup):
        step(k)
    drain()
    device_sync()
    st.synchronize()
    if dist:
        tdist.barrier()
    device_sync()
    t0 = time.perf_counter()
    c0 = time.process_time()
    for k in range(args.warmup, args.warmup + args.steps):
        step(k)
    c1 = time.process_time()
    drain()
    device_sync()
    st.synchronize()  # raises if any timed push's hand-off timed out
    if dist:
        tdist.barrier()
    el = time.perf_counter() - t0
    if dist:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        el = float(t.item())

    # exact check on rank 0: every rank's first and last stream of the last push
    verified, checked = None, []
    if rank == 0:
        last = (state["i"] - 1) % 2
        got = recvs[last] if dist else [packs[last].flat]
        verified = bool(torch.equal(got[0], packs[last].flat))
        for r in range(world):
            view = packs[last].views(S, flat=got[r])
            for b in sorted({0, S - 1}):
                g = r * S + b
                if args.stub:
                    exp = _StubStream.expect(g, state["i"])
                    ok = all(torch.equal(view[k][b], exp[k]) for k in KEYS)
                else:
                    a = stream_audio(g, n)  # every push so far, rolled into a zero window (run_sds.py:174,206-220)
                    w = np.zeros((1, 2, int(WINDOW_S * SR)), dtype=np.float32)
                    L = min(a.shape[1], w.shape[2])
                    w[0, :, w.shape[2] - L:] = a[:, a.shape[1] - L:]
                    win = torch.from_numpy(w).to(dev)
                    ref = m.probs(win)
                    ok = all(torch.equal(view[k][b], ref[k][0, -F:]) for k in KEYS)
                checked.append({"rank": r, "stream": g, "bit_identical": ok})
                verified = verified and ok
        if m is not None:
            m.synchronize()

    if rank == 0:
        B = world * S
        line = {"metric": "new audio-seconds/sec (whole node; streaming, 1 s hop / 10 s window)",
                "value": round(B * (HOP / SR) * args.steps / el, 1), "unit": "audio-s/s",
                "ms_per_step": round(el / args.steps * 1e3, 3), "n_gpus": world, "streams": B,
                "streams_per_gpu": S, "steps": args.steps, "warmup": args.warmup, "scaling": "weak",
                "reused_rows": st.reused_rows, "frames": st.frames, "dtype": args.precision,
                "data": "synthetic", "checked_each_push": args.check_each,
                "window_audio_s_per_s": round(B * WINDOW_S * args.steps / el, 1),
                "host_cpu_ms_per_push": round((c1 - c0) / args.steps * 1e3, 3), "graph": st.graph_info(),
                "config": f"BASELINE.json configs[4]: {B} streams ({S} per GPU x {world}), rolling 10 s window, "
                          f"1 s hop, hipGraph-replayed push",
                "gather": {"collective": "torch.distributed.gather" + (" (gloo)" if args.stub else " (RCCL)"),
                           "calls_per_step": 1 if dist else 0, "bytes_per_rank": packs[0].flat.numel() * 4,
                           "keys": list(KEYS), "overlapped_with_next_step": True, "verified": verified,
                           "clips_checked": checked}}
        print(json.dumps(line), flush=True)
    if dist:
        tdist.destroy_process_group()
    if rank == 0 and verified is not True:
        print("bench_stream.py: the gathered hop outputs failed the exact per-rank check", file=sys.stderr)
        return 3
    return 0


if __name__ == "__main__":
    sys.exit(main())
