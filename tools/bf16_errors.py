#!/usr/bin/env python3
"""Measure the bf16 perf path's max abs error against every reference fixture (tests/golden), per
output.  The bf16 tolerances in tests/test_gpu_parity.py are set from these numbers (<= 3x).

    python tools/bf16_errors.py > gpurun_out/bf16_errors.json      (GPU box)
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from vap.model import VapGPT  # noqa: E402
from voiceactivityprojection_amd.weights import synthetic_batch, synthetic_state_dict, synthetic_waveform  # noqa: E402

G = os.path.join(REPO, "tests", "golden")
KEYS = ("probs", "vad", "p_now", "p_future", "H", "loss")


def load(name):
    return dict(np.load(os.path.join(G, name + ".npz"), allow_pickle=False))


def main():
    precision = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    m = VapGPT(precision=precision)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed=0).items()}, strict=True)
    m = m.to("cuda").eval()
    cases = {
        "short_clip": lambda g: g["waveform"],
        "example_wav": lambda g: g["waveform"],
        "len_37392": lambda g: g["waveform"],
        "len_min": lambda g: g["waveform"],
        "batch_20s": lambda g: np.stack([synthetic_waveform(i, int(g["n_samples"])) for i in (0, 1)]),
        "bench4_20s": lambda g: synthetic_batch(0, 4, int(g["n_samples"])),
        "long_60s": lambda g: synthetic_waveform(int(g["clip_start"]), int(g["n_samples"]))[None],
        "len_320319": lambda g: synthetic_waveform(int(g["clip_start"]), int(g["n_samples"]))[None],
    }
    res = {}
    for name, mk in cases.items():
        g = load(name)
        out = m.probs(torch.from_numpy(mk(g)).cuda())
        m.synchronize()
        e = {}
        for k in KEYS:
            got = out[k].float().cpu().numpy()
            if k == "probs":
                if "probs" in g:
                    exp = g["probs"]
                elif "probs_stride10" in g:
                    got, exp = got[:, ::10], g["probs_stride10"]
                elif "probs_tail" in g:
                    got, exp = got[:, -g["probs_tail"].shape[1]:], g["probs_tail"]
                else:
                    continue
            else:
                exp = g[k]
            e[k] = float(np.abs(got - exp).max())
        res[name] = e
        print(name, e, file=sys.stderr, flush=True)
    res["max"] = {k: max(v.get(k, 0.0) for n, v in res.items()) for k in KEYS}
    print(json.dumps({"precision": precision, "errors": res}))


if __name__ == "__main__":
    main()
