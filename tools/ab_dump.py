#!/usr/bin/env python3
"""A/B bit-identity check: run VapGPT.probs (bf16) on a synthetic batch and save every output to an
npz; run once per library (VAP_LIB_AB=<name>.so) and compare the files with --compare.

    VAP_LIB_AB=x.so python tools/ab_dump.py --out gpurun_out/x.npz [--batch 16 --seconds 20]
    python tools/ab_dump.py --compare gpurun_out/a.npz gpurun_out/b.npz
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--compare", nargs=2)
    a = ap.parse_args()
    if a.compare:
        x, y = np.load(a.compare[0]), np.load(a.compare[1])
        keys = [k for k in x.files if not k.endswith("_sub")]
        bad = [k for k in keys if x[k] != y[k]]
        for k in keys:
            d = np.abs(x[k + "_sub"] - y[k + "_sub"]).max()
            print(k, "identical" if k not in bad else f"DIFFERS (subsample max {d:.3g})")
        sys.exit(1 if bad else 0)
    import torch
    from vap.model import VapGPT
    from voiceactivityprojection_amd.weights import synthetic_batch, synthetic_state_dict

    sd = synthetic_state_dict(seed=0)
    m = VapGPT(precision="bf16")
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    m = m.to("cuda:0").eval()
    n = int(a.seconds * 16000)
    wav = torch.from_numpy(synthetic_batch(0, a.batch, n)).to("cuda:0")
    out = m.probs(wav)
    torch.cuda.synchronize()
    # per output: a digest of the exact bytes (bit identity) and a subsample (size of a difference)
    import hashlib
    res = {}
    for k, v in out.items():
        arr = np.ascontiguousarray(v.float().cpu().numpy())
        res[k] = np.array(hashlib.sha256(arr.tobytes()).hexdigest())
        res[k + "_sub"] = arr.reshape(arr.shape[0], -1)[:, ::97]
    np.savez(a.out, **res)
    print("saved", a.out, {k: tuple(v.shape) for k, v in out.items()})


if __name__ == "__main__":
    main()
