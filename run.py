#!/usr/bin/env python3
"""CLI mirror of the reference run.py (run.py:134-279) on the MI355X engine.

    python run.py -a example.wav [-f out.json] [-sd state_dict.pt | -sd synthetic] [--chunk] [--vap_* ...]

Same flags, same JSON output (keys probs, vad, p_now, p_future, H, loss as nested lists; file name =
wav basename .json).  Differences, by design:
  * ``-sd synthetic`` loads the deterministic synthetic weights (the reference ships none);
  * ``step_extraction`` runs every fold of the long-audio chunking as ONE batched probs() call
    (folds are independent clips; outputs are identical to the reference's per-fold loop because
    the engine is batch-invariant).  Like the reference (quirk Q4) ``--chunk_time/--step_time`` are
    ignored and 20 s context + 5 s step are used, unless ``--honor_chunk_args`` is given.
"""
from __future__ import annotations

import os
import sys
from argparse import ArgumentParser
from os.path import basename

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from vap.model import VapConfig, VapGPT  # noqa: E402
from voiceactivityprojection_amd.audio import load_waveform  # noqa: E402
from voiceactivityprojection_amd.utils import batch_to_device, tensor_dict_to_json, write_json  # noqa: E402

OUT_KEYS = ("vad", "p_now", "p_future", "probs", "H")


def step_extraction(waveform, model, device="cpu", context_time=20, step_time=5, fold_batch=16, **_):
    """Long-audio extraction (run.py:23-131): context+step windows, first fold kept whole, every
    later fold contributes its last step_frames, tail fold covers the remainder; "loss" is the first
    fold's, as in the reference.

    All folds are processed in batches of ``fold_batch`` clips per probs() call."""
    n_samples = waveform.shape[-1]
    duration = round(n_samples / model.sample_rate, 2)
    chunk_time = context_time + step_time
    step_samples = int(step_time * model.sample_rate)
    chunk_samples = int(chunk_time * model.sample_rate)
    step_frames = int(step_time * model.frame_hz)
    folds = waveform.unfold(dimension=-1, size=chunk_samples, step=step_samples).permute(2, 0, 1, 3)
    expected_frames = round(duration * model.frame_hz)

    B = waveform.shape[0]
    flat = folds.reshape(-1, 2, chunk_samples)  # (n_folds * B, 2, chunk)
    parts = {k: [] for k in OUT_KEYS + ("loss",)}
    for i in range(0, flat.shape[0], fold_batch * B):
        o = model.probs(flat[i: i + fold_batch * B].to(device))
        for k in parts:
            parts[k].append(o[k])
    allo = {k: torch.cat(v, 0).view(folds.shape[0], B, *v[0].shape[1:]) for k, v in parts.items()}
    out = {k: torch.cat([allo[k][0]] + [allo[k][f][:, -step_frames:] for f in range(1, folds.shape[0])], dim=1)
           for k in OUT_KEYS}
    # the reference's `out` starts as the first fold's probs() dict and only the OUT_KEYS grow, so
    # the first fold's "loss" (B, chunk_frames - horizon) stays in it and reaches the JSON (run.py:66)
    out["loss"] = allo["loss"][0]
    processed = out["p_now"].shape[1]
    if expected_frames != processed:
        omitted = expected_frames - processed
        o = model.probs(waveform[..., -chunk_samples:].to(device))
        for k in OUT_KEYS:
            out[k] = torch.cat([out[k], o[k][:, -omitted:]], dim=1)
    model.synchronize()  # raises if a recurrence hand-off timed out (the outputs would be invalid)
    return batch_to_device(out, "cpu")


def get_args(argv=None):
    parser = ArgumentParser()
    parser.add_argument("-a", "--audio", type=str, help="Path to waveform")
    parser.add_argument("-f", "--filename", type=str, default=None, help="Path to waveform")
    parser.add_argument("-sd", "--state_dict", type=str,
                        default="example/VAP_3mmz3t0u_50Hz_ad20s_134-epoch9-val_2.56.pt",
                        help="Path to state_dict ('synthetic' = deterministic synthetic weights)")
    parser.add_argument("-c", "--checkpoint", type=str, default=None, help="Path to trained model")
    parser, _ = VapConfig.add_argparse_args(parser)
    parser.add_argument("--chunk", action="store_true",
                        help="Process the audio in chunks (longer > 164s on 24Gb GPU audio)")
    parser.add_argument("--chunk_time", type=float, default=30, help="Duration of each chunk processed by model")
    parser.add_argument("--step_time", type=float, default=5, help="Increment to process in a step")
    parser.add_argument("--honor_chunk_args", action="store_true",
                        help="use --chunk_time/--step_time (the reference ignores them: 20 s context + 5 s step)")
    parser.add_argument("--precision", default=os.environ.get("VAP_PRECISION", "fp32"), choices=["fp32", "bf16"])
    parser.add_argument("--plot", action="store_true", help="Visualize output (matplotlib)")
    args = parser.parse_args(argv)
    conf = VapConfig.args_to_conf(args)
    return args, conf


def load_model(args, conf) -> VapGPT:
    model = VapGPT(conf, precision=args.precision)
    if args.checkpoint is not None:
        raise NotImplementedError("Not implemeted from checkpoint...")  # reference run.py:202-207
    if args.state_dict != "synthetic":
        sd = torch.load(args.state_dict, map_location="cpu", weights_only=True)
        model.load_state_dict(sd)
    return model


def main(argv=None):
    args, conf = get_args(argv)
    print("Load Model...")
    model = load_model(args, conf)
    device = "cuda" if torch.cuda.is_available() else "cpu"
    model = model.to(device).eval()

    waveform, _ = load_waveform(args.audio, sample_rate=model.sample_rate)
    duration = round(waveform.shape[-1] / model.sample_rate)
    if waveform.shape[0] == 1:
        waveform = torch.cat((waveform, torch.zeros_like(waveform)))
    waveform = waveform.unsqueeze(0)
    if duration > 160:
        print(f"WARNING: {duration} > 160s: using chunked extraction")
        args.chunk = True

    if args.chunk:
        ctx, step = (args.chunk_time - args.step_time, args.step_time) if args.honor_chunk_args else (20, 5)
        out = step_extraction(waveform, model, device, context_time=ctx, step_time=step)
    else:
        out = model.probs(waveform.to(device))
        model.synchronize()  # raises if a recurrence hand-off timed out (the outputs would be invalid)
        out = batch_to_device(out, "cpu")

    for k, v in out.items():
        if isinstance(v, torch.Tensor):
            print(f"{k}: ", tuple(v.shape))
    if args.filename is None:
        args.filename = basename(args.audio).replace(".wav", ".json")
    if not args.filename.endswith(".json"):
        args.filename += ".json"
    write_json(tensor_dict_to_json(out), args.filename)
    print("wavefile: ", args.audio)
    print("Saved output -> ", args.filename)
    return out


if __name__ == "__main__":
    main()
