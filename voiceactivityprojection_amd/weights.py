"""State-dict schema of the VAP model and deterministic synthetic weights / waveforms.

The reference ships no weights (``/root/reference/.MISSING_LARGE_BLOBS:1,5-7``), so every parity
fixture and every benchmark runs on *synthetic* weights.  They come from a counter-based generator
(splitmix64 over a per-key stream) that is identical here, on the GPU box and inside
``tools/gen_golden.py`` (which loads them into the reference's own ``VapGPT``), so no 23 MB blob has
to travel.

Schema follows the reference module tree:
  * ``vap/model.py:125-163``          VapGPT (encoder, ar_channel, ar, objective, heads)
  * ``vap/encoder.py:16-31``          EncoderCPC (encoder = CPCModel, downsample = get_cnn_layer)
  * ``vap/encoder_components.py:73-176,485-499``  CPCEncoder / CPCAR / CConv1d / LayerNorm
  * ``vap/modules.py:113-449``        MultiHeadAttentionAlibi / TransformerLayer / GPT / Combinator
  * ``vap/objective.py:79-110``       Codebook.emb (fixed code vectors)
"""
from __future__ import annotations

import hashlib
import math
from typing import Dict, List, Tuple

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    """Vectorised splitmix64 finaliser (wrapping uint64 arithmetic)."""
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def _stream_seed(tag: str, seed: int) -> np.uint64:
    h = hashlib.sha256(f"{seed}:{tag}".encode()).digest()
    return np.uint64(int.from_bytes(h[:8], "little"))


def uniform(tag: str, n: int, seed: int = 0) -> np.ndarray:
    """n float32 values uniform in [-1, 1), exactly reproducible (24-bit mantissa grid)."""
    base = _stream_seed(tag, seed)
    with np.errstate(over="ignore"):
        ctr = base + np.arange(n, dtype=np.uint64) * np.uint64(0xD1B54A32D192ED03)
    bits = _splitmix64(ctr) >> np.uint64(40)  # 24 random bits
    return (bits.astype(np.float64) / float(1 << 23) - 1.0).astype(np.float32)


def normal(tag: str, n: int, seed: int = 0) -> np.ndarray:
    """n float32 standard normals (Box-Muller over two counter streams), reproducible."""
    base = _stream_seed(tag, seed)
    with np.errstate(over="ignore"):
        ctr = base + np.arange(n, dtype=np.uint64) * np.uint64(2) * np.uint64(0xD1B54A32D192ED03)
        u1 = (_splitmix64(ctr) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))
        u2 = (_splitmix64(ctr + np.uint64(0xD1B54A32D192ED03)) >> np.uint64(11)).astype(np.float64) * (
            1.0 / (1 << 53)
        )
    u1 = np.maximum(u1, 1e-300)
    return (np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * math.pi * u2)).astype(np.float32)


def alibi_slopes(n: int) -> List[float]:
    """AliBi head slopes, restating ``MultiHeadAttentionAlibi.get_slopes`` (vap/modules.py:124-158)."""

    def pow2(n):
        start = 2 ** (-(2 ** -(math.log2(n) - 3)))
        return [start * start**i for i in range(n)]

    if math.log2(n).is_integer():
        return pow2(n)
    c = 2 ** math.floor(math.log2(n))
    return pow2(c) + alibi_slopes(2 * c)[0::2][: n - c]


def code_vectors(n_bins_total: int) -> np.ndarray:
    """Codebook.create_code_vectors (vap/objective.py:101-110): row k = bits of k, LSB first."""
    k = np.arange(2**n_bins_total)[:, None]
    return ((k >> np.arange(n_bins_total)[None, :]) & 1).astype(np.float32)


def bin_frames(bin_times, frame_hz) -> List[int]:
    """bin_times_to_frames (vap/objective.py:10-11): float32 product truncated to int."""
    return [int(v) for v in (np.asarray(bin_times, dtype=np.float32) * np.float32(frame_hz)).astype(np.int64)]


def schema(dim: int = 256, channel_layers: int = 1, cross_layers: int = 3, num_heads: int = 4,
           lstm_layers: int = 1, n_bins: int = 4, cpc_dim: int = 256, mono: bool = False,
           va_history_bins: int = 0) -> List[Tuple[str, Tuple[int, ...]]]:
    """Ordered (key, shape) list == ``VapGPT(conf).state_dict()`` of the reference, or with ``mono``
    ``VapGPTMono(VapMonoConfig(va_history=va_history_bins > 0)).state_dict()`` (vap/model.py:271-323)."""
    C = cpc_dim
    out: List[Tuple[str, Tuple[int, ...]]] = []
    g = "encoder.encoder.gEncoder"
    conv_specs = [(1, 10), (C, 8), (C, 4), (C, 4), (C, 4)]  # encoder_components.py:83-92
    for i, (cin, k) in enumerate(conv_specs):
        out += [(f"{g}.conv{i}.weight", (C, cin, k)), (f"{g}.conv{i}.bias", (C,)),
                (f"{g}.batchNorm{i}.weight", (1, C, 1)), (f"{g}.batchNorm{i}.bias", (1, C, 1))]
    for l in range(lstm_layers):  # encoder_components.py:123-126 (nn.LSTM)
        p = "encoder.encoder.gAR.baseNet"
        out += [(f"{p}.weight_ih_l{l}", (4 * C, C)), (f"{p}.weight_hh_l{l}", (4 * C, C)),
                (f"{p}.bias_ih_l{l}", (4 * C,)), (f"{p}.bias_hh_l{l}", (4 * C,))]
    out += [("encoder.downsample.1.weight", (C, C, 5)), ("encoder.downsample.1.bias", (C,)),
            ("encoder.downsample.2.ln.weight", (C,)), ("encoder.downsample.2.ln.bias", (C,))]
    dff = 3 * dim

    def layer(prefix, cross):
        r = [(f"{prefix}.ln_self_attn.weight", (dim,)), (f"{prefix}.ln_self_attn.bias", (dim,)),
             (f"{prefix}.ln_ffnetwork.weight", (dim,)), (f"{prefix}.ln_ffnetwork.bias", (dim,)),
             (f"{prefix}.mha.m", (num_heads,))]
        r += [(f"{prefix}.mha.{n}.weight", (dim, dim)) for n in ("key", "query", "value", "proj")]
        r += [(f"{prefix}.ffnetwork.0.weight", (dff, dim)), (f"{prefix}.ffnetwork.3.weight", (dim, dff))]
        if cross:
            r += [(f"{prefix}.ln_src_attn.weight", (dim,)), (f"{prefix}.ln_src_attn.bias", (dim,)),
                  (f"{prefix}.mha_cross.m", (num_heads,))]
            r += [(f"{prefix}.mha_cross.{n}.weight", (dim, dim)) for n in ("key", "query", "value", "proj")]
        return r

    nb = 2 * n_bins
    if mono:  # init_va_conditioning (model.py:317-323), plain GPT stacks, vap_head
        out += [("va_condition.weight", (dim, 2)), ("va_condition.bias", (dim,)),
                ("va_cond_ln.weight", (dim,)), ("va_cond_ln.bias", (dim,))]
        if va_history_bins:
            out += [("va_cond_history.weight", (dim, va_history_bins)), ("va_cond_history.bias", (dim,))]
        for l in range(channel_layers):
            out += layer(f"ar_channel.layers.{l}", False)
        for l in range(cross_layers):
            out += layer(f"ar.layers.{l}", False)
        out += [("objective.codebook.emb.weight", (2**nb, nb)),
                ("vap_head.weight", (2**nb, dim)), ("vap_head.bias", (2**nb,))]
        return out
    for l in range(channel_layers):
        out += layer(f"ar_channel.layers.{l}", False)
    for l in range(cross_layers):
        out += layer(f"ar.layers.{l}", True)
    out += [("ar.combinator.h0_a.weight", (dim, dim)), ("ar.combinator.h0_b.weight", (dim, dim)),
            ("ar.combinator.ln.weight", (dim,)), ("ar.combinator.ln.bias", (dim,))]
    nb = 2 * n_bins
    out += [("objective.codebook.emb.weight", (2**nb, nb)),
            ("va_classifier.weight", (1, dim)), ("va_classifier.bias", (1,)),
            ("vap_head.weight", (2**nb, dim)), ("vap_head.bias", (2**nb,))]
    return out


def _fan_in(key: str, shape) -> int:
    if len(shape) == 3:
        return shape[1] * shape[2]
    if len(shape) == 2:
        return shape[1]
    return 256


def synthetic_state_dict(seed: int = 0, **schema_kw) -> Dict[str, np.ndarray]:
    """Deterministic float32 weights for every key of :func:`schema`.

    Scales: PyTorch-default-like ``U(-1/sqrt(fan_in), 1/sqrt(fan_in))`` for conv/LSTM/Linear weights
    and biases, with ``sqrt(3)`` gain on attention/FFN/head Linears so attention scores are not
    uniform; norm affine params perturbed away from 1/0; AliBi slopes and the
    codebook are the reference's fixed values.
    """
    sd: Dict[str, np.ndarray] = {}
    heads = schema_kw.get("num_heads", 4)
    shapes = dict(schema(**schema_kw))
    for key, shape in schema(**schema_kw):
        n = int(np.prod(shape))
        leaf = key.rsplit(".", 1)[-1]
        if key.endswith(".m"):
            v = np.asarray(alibi_slopes(heads), dtype=np.float32)
        elif key == "objective.codebook.emb.weight":
            v = code_vectors(shape[1])
        elif ("batchNorm" in key or ".ln" in key or "ln_" in key or "_ln." in key) and leaf == "weight":
            v = 1.0 + 0.2 * uniform(key, n, seed)
        elif ("batchNorm" in key or ".ln" in key or "ln_" in key or "_ln." in key) and leaf == "bias":
            v = 0.1 * uniform(key, n, seed)
        elif "gAR" in key:
            v = uniform(key, n, seed) / np.float32(16.0)  # nn.LSTM default U(-1/sqrt(H), 1/sqrt(H))
        elif leaf == "bias":
            wshape = shapes.get(key[: -len("bias")] + "weight", (n, 256))
            v = uniform(key, n, seed) / np.float32(math.sqrt(_fan_in(key, wshape)))
        else:
            gain = 1.0 if ("gEncoder" in key or "downsample" in key) else math.sqrt(3.0)
            v = uniform(key, n, seed) * np.float32(gain / math.sqrt(_fan_in(key, shape)))
        sd[key] = np.ascontiguousarray(v.reshape(shape).astype(np.float32))
    return sd


def synthetic_waveform(clip_index: int, n_samples: int, channels: int = 2, std: float = 0.1) -> np.ndarray:
    """Stereo clip ``(channels, n_samples)`` float32: N(0, std^2) clipped to [-1, 1].

    Seed = 1234 + global clip index, so data-parallel shards are reproducible.
    """
    x = normal(f"wave:{1234 + clip_index}", channels * n_samples, seed=0) * np.float32(std)
    return np.clip(x, -1.0, 1.0).reshape(channels, n_samples)


def synthetic_batch(start: int, batch: int, n_samples: int) -> np.ndarray:
    return np.stack([synthetic_waveform(start + b, n_samples) for b in range(batch)])
