"""ORACLE — test infrastructure only, never the product path.

CPU fp32 restatement of the reference VAP forward + ``probs()`` path
(ErikEkstedt/VoiceActivityProjection @ /root/reference), written as plain functions over a
state dict.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as the checker / CPU baseline.  The shipped engine
(``voiceactivityprojection_amd``) never imports it and fails loudly without its HIP library.

Pinning: ``tests/test_oracle_golden.py`` checks every function here against golden vectors that
``tools/gen_golden.py`` produced by importing the reference's own ``vap.model.VapGPT`` in the build
container; the label / frame-length code is integer arithmetic and is pinned
bit-exactly.

Floating point follows the reference's ATen op sequence (conv1d, LSTM, layer_norm, softmax,
einsum) so the noise floor vs the reference is ~1e-7 (SURVEY.md §8(c) "Oracle noise floor").
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

Tensor = torch.Tensor
SD = Dict[str, Tensor]


# --------------------------------------------------------------------------------------------
# A1 frame-length chain
# --------------------------------------------------------------------------------------------
def conv_out_len(n: int, k: int, s: int, p_left: int, p_right: int) -> int:
    return (n + p_left + p_right - k) // s + 1


def frame_lengths(n_samples: int) -> List[int]:
    """Lengths after conv0..conv4 (encoder_components.py:83-92) and the causal stride-2
    downsample (CConv1d pad (4,0), encoder_components.py:454-460, encoder.py:24-31)."""
    a0 = conv_out_len(n_samples, 10, 5, 3, 3)
    a1 = conv_out_len(a0, 8, 4, 2, 2)
    a2 = conv_out_len(a1, 4, 2, 1, 1)
    a3 = conv_out_len(a2, 4, 2, 1, 1)
    a4 = conv_out_len(a3, 4, 2, 1, 1)
    t = conv_out_len(a4, 5, 2, 4, 0)
    return [a0, a1, a2, a3, a4, t]


# --------------------------------------------------------------------------------------------
# A3-A5 CPC encoder
# --------------------------------------------------------------------------------------------
def channel_norm(x: Tensor, w: Tensor, b: Tensor, eps: float = 1e-5) -> Tensor:
    """ChannelNorm.forward (encoder_components.py:62-70): mean and UNBIASED var over dim 1."""
    mu = x.mean(dim=1, keepdim=True)
    var = x.var(dim=1, keepdim=True)
    return (x - mu) * torch.rsqrt(var + eps) * w + b


_CONV_SPECS = [(10, 5, 3), (8, 4, 2), (4, 2, 1), (4, 2, 1), (4, 2, 1)]  # encoder_components.py:83-92


def cpc_encoder(wav: Tensor, sd: SD, taps: Optional[dict] = None) -> Tensor:
    """CPCEncoder.forward (encoder_components.py:98-104): 5x [conv -> ChannelNorm -> ReLU].
    wav (B, 1, N) -> (B, 256, a4)."""
    g = "encoder.encoder.gEncoder"
    x = wav
    for i, (k, s, p) in enumerate(_CONV_SPECS):
        x = F.conv1d(x, sd[f"{g}.conv{i}.weight"], sd[f"{g}.conv{i}.bias"], stride=s, padding=p)
        x = F.relu(channel_norm(x, sd[f"{g}.batchNorm{i}.weight"], sd[f"{g}.batchNorm{i}.bias"]))
        if taps is not None:
            taps[f"conv{i}"] = x
    return x


def lstm_layers(sd: SD) -> int:
    n = 0
    while f"encoder.encoder.gAR.baseNet.weight_ih_l{n}" in sd:
        n += 1
    return n


def lstm(x: Tensor, sd: SD) -> Tensor:
    """CPCAR.forward (encoder_components.py:140-159) -> nn.LSTM(batch_first, zero init state,
    no reverse, no keepHidden; config :380-391). Gates i,f,g,o (PyTorch order).
    x (B, T, 256) -> (B, T, 256)."""
    p = "encoder.encoder.gAR.baseNet"
    L = lstm_layers(sd)
    H = sd[f"{p}.weight_hh_l0"].shape[1]
    mod = torch.nn.LSTM(x.shape[-1], H, num_layers=L, batch_first=True)
    with torch.no_grad():
        for l in range(L):
            for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh"):
                getattr(mod, f"{n}_l{l}").copy_(sd[f"{p}.{n}_l{l}"])
        y, _ = mod(x)
    return y


def lstm_loop(x: Tensor, sd: SD) -> Tensor:
    """Same recurrence written out step by step (documents the math the HIP kernel implements):
    z = x W_ih^T + b_ih + h W_hh^T + b_hh; i,f,g,o = split(z); c = sig(f) c + sig(i) tanh(g);
    h = sig(o) tanh(c)."""
    p = "encoder.encoder.gAR.baseNet"
    for l in range(lstm_layers(sd)):
        wih, whh = sd[f"{p}.weight_ih_l{l}"], sd[f"{p}.weight_hh_l{l}"]
        b = sd[f"{p}.bias_ih_l{l}"] + sd[f"{p}.bias_hh_l{l}"]
        B, T, _ = x.shape
        H = whh.shape[1]
        gx = x @ wih.T + b
        h = x.new_zeros(B, H)
        c = x.new_zeros(B, H)
        ys = []
        for t in range(T):
            z = gx[:, t] + h @ whh.T
            i, f, g, o = z.split(H, dim=-1)
            c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
            h = torch.sigmoid(o) * torch.tanh(c)
            ys.append(h)
        x = torch.stack(ys, dim=1)
    return x


def downsample(x: Tensor, sd: SD) -> Tensor:
    """get_cnn_layer (encoder_components.py:485-499): rearrange -> CConv1d(k5, s2, left pad 4,
    :454-460) -> LayerNorm over channels (:405-425, biased var, eps 1e-5) -> GELU(erf).
    (B, T2, 256) -> (B, T, 256)."""
    z = x.transpose(1, 2)
    z = F.pad(z, (4, 0))
    z = F.conv1d(z, sd["encoder.downsample.1.weight"], sd["encoder.downsample.1.bias"], stride=2)
    z = z.transpose(1, 2)
    z = F.layer_norm(z, (z.shape[-1],), sd["encoder.downsample.2.ln.weight"], sd["encoder.downsample.2.ln.bias"])
    return F.gelu(z)


def encoder(wav1: Tensor, sd: SD, taps: Optional[dict] = None) -> Tensor:
    """EncoderCPC.forward (encoder.py:49-66). wav1 (B, N) or (B, 1, N) -> (B, T, 256)."""
    if wav1.ndim < 3:
        wav1 = wav1.unsqueeze(1)
    z = cpc_encoder(wav1, sd, taps)
    z = z.transpose(1, 2)
    z = lstm(z, sd)
    if taps is not None:
        taps["lstm"] = z
    return downsample(z, sd)


# --------------------------------------------------------------------------------------------
# A8-A14 transformer
# --------------------------------------------------------------------------------------------
def alibi_bias(T: int, m: Tensor, Tk: Optional[int] = None) -> Tensor:
    """MultiHeadAttentionAlibi.get_alibi_mask (modules.py:169-187): bias[h,i,j] = m_h * j for j <= i,
    -inf above the diagonal. Shape (1, H, T, T)."""
    Tk = T if Tk is None else Tk
    rel = torch.arange(Tk, dtype=torch.float32).view(1, 1, -1) * m.view(1, -1, 1)  # (1,H,Tk)
    causal = torch.tril(torch.ones(T, Tk))
    mask = torch.zeros(T, Tk).masked_fill(causal == 0, float("-inf"))
    return rel.unsqueeze(-2) + mask


def mha(Q: Tensor, K: Tensor, V: Tensor, sd: SD, prefix: str, num_heads: int, maps: Optional[list] = None) -> Tensor:
    """MultiHeadAttention.forward (modules.py:82-110) with the AliBi mask (modules.py:189-202).
    Linear projections without bias (:38-40,51); scale = 1/sqrt(dim) (:52, Q5).  ``maps`` collects
    the softmax weights (B, H, T, T) the reference returns as ``att`` (:110)."""
    B, T, D = Q.shape
    h = num_heads

    def heads(x):
        return x.view(B, T, h, D // h).transpose(1, 2)

    k = heads(K @ sd[f"{prefix}.key.weight"].T)
    q = heads(Q @ sd[f"{prefix}.query.weight"].T)
    v = heads(V @ sd[f"{prefix}.value.weight"].T)
    att = torch.einsum("bhid,bhjd->bhij", q, k) * (1.0 / math.sqrt(D))
    att = att + alibi_bias(T, sd[f"{prefix}.m"])
    att = F.softmax(att, dim=-1)
    if maps is not None:
        maps.append(att)
    y = (att @ v).transpose(1, 2).reshape(B, T, D)
    return y @ sd[f"{prefix}.proj.weight"].T


def layer_norm(x: Tensor, sd: SD, prefix: str) -> Tensor:
    return F.layer_norm(x, (x.shape[-1],), sd[f"{prefix}.weight"], sd[f"{prefix}.bias"])


def transformer_layer(x: Tensor, sd: SD, prefix: str, num_heads: int, src: Optional[Tensor] = None,
                      smaps: Optional[list] = None, cmaps: Optional[list] = None) -> Tensor:
    """TransformerLayer.forward (modules.py:246-275), eval mode (dropout = identity).
    Pre-LN self-attn + residual; cross-attn Q = LN_src(x), K = V = raw src (:265-272); FFN
    (ffn_block :9-21: Linear -> GELU -> Linear, no bias) + residual."""
    z = layer_norm(x, sd, f"{prefix}.ln_self_attn")
    x = x + mha(z, z, z, sd, f"{prefix}.mha", num_heads, smaps)
    if src is not None:
        z = layer_norm(x, sd, f"{prefix}.ln_src_attn")
        x = x + mha(z, src, src, sd, f"{prefix}.mha_cross", num_heads, cmaps)
    z = layer_norm(x, sd, f"{prefix}.ln_ffnetwork")
    z = F.gelu(z @ sd[f"{prefix}.ffnetwork.0.weight"].T) @ sd[f"{prefix}.ffnetwork.3.weight"].T
    return x + z


def count_layers(sd: SD, prefix: str) -> int:
    n = 0
    while f"{prefix}.layers.{n}.ln_self_attn.weight" in sd:
        n += 1
    return n


def gpt(x: Tensor, sd: SD, num_heads: int, smaps: Optional[list] = None) -> Tensor:
    """GPT.forward (modules.py:342-358) for ``ar_channel``."""
    for l in range(count_layers(sd, "ar_channel")):
        x = transformer_layer(x, sd, f"ar_channel.layers.{l}", num_heads, smaps=smaps)
    return x


def combinator(x1: Tensor, x2: Tensor, sd: SD) -> Tensor:
    """Combinator.forward (modules.py:434-449): one shared LN, GELU, no biases."""
    ha = F.gelu(layer_norm(x1 @ sd["ar.combinator.h0_a.weight"].T, sd, "ar.combinator.ln"))
    hb = F.gelu(layer_norm(x2 @ sd["ar.combinator.h0_b.weight"].T, sd, "ar.combinator.ln"))
    return ha + hb


def gpt_stereo(x1: Tensor, x2: Tensor, sd: SD, num_heads: int, maps: Optional[dict] = None):
    """GPTStereo.forward (modules.py:380-408) + TransformerStereoLayer (:279-289): both towers use
    the PRE-layer x1/x2 as each other's src.  ``maps`` collects the per-layer weights of each tower
    under "sa" / "ca" (self / cross) as lists [tower a, tower b]."""
    m = maps if maps is not None else {"sa": [[], []], "ca": [[], []]}
    for l in range(count_layers(sd, "ar")):
        p = f"ar.layers.{l}"
        z1 = transformer_layer(x1, sd, p, num_heads, src=x2, smaps=m["sa"][0], cmaps=m["ca"][0])
        z2 = transformer_layer(x2, sd, p, num_heads, src=x1, smaps=m["sa"][1], cmaps=m["ca"][1])
        x1, x2 = z1, z2
    return combinator(x1, x2, sd), x1, x2


# --------------------------------------------------------------------------------------------
# A15-A20 model forward / probs / objective
# --------------------------------------------------------------------------------------------
def forward(waveform: Tensor, sd: SD, num_heads: int = 4, taps: Optional[dict] = None,
            attention: bool = False) -> Dict[str, Tensor]:
    """VapGPT.forward (model.py:249-268). waveform (B, 2, N) -> logits (B,T,256), vad (B,T,2); with
    ``attention`` also self_attn (B,2,Lc,H,T,T), cross_attn / cross_self_attn (B,2,Lx,H,T,T)
    (model.py:264-267, modules.py:349-356 / 400-407)."""
    assert waveform.shape[1] == 2, f"audio VAP ENCODER: {waveform.shape} != (B, 2, n_samples)"
    x1 = encoder(waveform[:, :1], sd, taps)  # model.py:173-174
    x2 = encoder(waveform[:, 1:], sd, None)
    if taps is not None:
        taps["enc1"], taps["enc2"] = x1, x2
    s1, s2 = [], []
    o1 = gpt(x1, sd, num_heads, s1)
    o2 = gpt(x2, sd, num_heads, s2)
    if taps is not None:
        taps["ar_channel1"], taps["ar_channel2"] = o1, o2
    maps = {"sa": [[], []], "ca": [[], []]}
    x, y1, y2 = gpt_stereo(o1, o2, sd, num_heads, maps)
    w, b = sd["va_classifier.weight"], sd["va_classifier.bias"]
    vad = torch.cat((y1 @ w.T + b, y2 @ w.T + b), dim=-1)
    logits = x @ sd["vap_head.weight"].T + sd["vap_head.bias"]
    ret = {"logits": logits, "vad": vad}
    if attention:
        def stk(a, b):  # per tower: layers stacked on dim 1, then towers on dim 1
            return torch.stack([torch.stack(a, dim=1), torch.stack(b, dim=1)], dim=1)
        ret["self_attn"] = stk(s1, s2)
        ret["cross_attn"] = stk(*maps["ca"])
        ret["cross_self_attn"] = stk(*maps["sa"])
    return ret


def aggregate_matrix(n_bins: int, from_bin: int, to_bin: int) -> Tensor:
    """abp[k, c] = sum_{b=from..to} bit(c*n_bins + b) of k (objective.py:184-204, 101-110, 141-143)."""
    nc = 2 ** (2 * n_bins)
    k = torch.arange(nc).view(-1, 1, 1)
    c = torch.arange(2).view(1, -1, 1)
    bb = torch.arange(n_bins).view(1, 1, -1)
    states = ((k >> (c * n_bins + bb)) & 1).float()  # (nc, 2, n_bins)
    return states[:, :, from_bin: to_bin + 1].sum(-1)


def probs_next_speaker_aggregate(probs: Tensor, from_bin: int, to_bin: int, n_bins: int = 4) -> Tensor:
    """ObjectiveVAP.probs_next_speaker_aggregate (objective.py:184-204)."""
    abp = aggregate_matrix(n_bins, from_bin, to_bin)
    p_all = torch.einsum("bid,dc->bic", probs, abp)
    return p_all / (p_all.sum(-1, keepdim=True) + 1e-5)


def get_labels_np(va: np.ndarray, bin_frames: List[int], threshold: float = 0.5) -> np.ndarray:
    """ObjectiveVAP.get_labels (objective.py:209-212) = ProjectionWindow (:40-76) + Codebook.encode
    (:112-139), restated as integer bit packing: window = va[:, 1:] unfolded over sum(bin_frames);
    bit(c, b) = (sum over bin b of channel c) / len_b >= threshold (float32 arithmetic, as the
    reference); label = sum bit(c,b) * 2^(c*n_bins + b).  va (B, T, 2) float -> (B, T - horizon) int64.

    Raises RuntimeError when T - 1 < horizon (reference quirk Q2, ``unfold`` size error)."""
    va = np.asarray(va, dtype=np.float32)
    B, T, C = va.shape
    horizon = int(sum(bin_frames))
    n = T - 1 - horizon + 1
    if n <= 0:
        raise RuntimeError(
            f"maximum size for tensor at dimension 1 is {T - 1} but size is {horizon}")
    nb = len(bin_frames)
    labels = np.zeros((B, n), dtype=np.int64)
    start = 0
    for bi, bf in enumerate(bin_frames):
        # cumulative sums in float64 are exact for binary VA; for soft VA we sum in float32 order
        win = np.stack([va[:, 1 + start + j: 1 + start + j + n, :] for j in range(bf)], axis=0)
        s = np.zeros((B, n, C), dtype=np.float32)
        for j in range(bf):
            s = (s + win[j]).astype(np.float32)
        ratio = (s / np.float32(bf)).astype(np.float32)
        bits = (ratio >= np.float32(threshold)).astype(np.int64)
        for c in range(C):
            labels += bits[..., c] << (c * nb + bi)
        start += bf
    return labels


def label_ratios_np(va: np.ndarray, bin_frames: List[int]) -> np.ndarray:
    """Per (b, t, c, bin) activity ratios (float64), used by tests to skip frames whose ratio is
    within rounding distance of the 0.5 threshold."""
    va = np.asarray(va, dtype=np.float64)
    B, T, C = va.shape
    horizon = int(sum(bin_frames))
    n = T - horizon
    out = np.zeros((B, n, C, len(bin_frames)))
    start = 0
    for bi, bf in enumerate(bin_frames):
        acc = np.zeros((B, n, C))
        for j in range(bf):
            acc += va[:, 1 + start + j: 1 + start + j + n, :]
        out[..., bi] = acc / bf
        start += bf
    return out


def loss_vap(logits: Tensor, labels: Tensor) -> Tensor:
    """ObjectiveVAP.loss_vap(reduction='none') (objective.py:220-243)."""
    nmax = labels.shape[1]
    lg = logits[:, :nmax]
    loss = F.cross_entropy(lg.reshape(-1, lg.shape[-1]), labels.reshape(-1), reduction="none")
    return loss.view(-1, nmax)


def probs(waveform: Tensor, sd: SD, num_heads: int = 4, bin_frames: Optional[List[int]] = None,
          now_lims=(0, 1), future_lims=(2, 3), taps: Optional[dict] = None) -> Dict[str, Tensor]:
    """VapGPT.probs (model.py:180-225) including quirk Q1 (labels from the model's own sigmoid
    VAD, so ``loss`` is always returned)."""
    bin_frames = [10, 20, 30, 40] if bin_frames is None else bin_frames
    nb = len(bin_frames)
    with torch.no_grad():
        out = forward(waveform, sd, num_heads, taps)
        pr = out["logits"].softmax(dim=-1)
        vad = out["vad"].sigmoid()
        H = (-pr * pr.log2()).sum(dim=-1)
        p_now = probs_next_speaker_aggregate(pr, now_lims[0], now_lims[-1], nb)
        p_future = probs_next_speaker_aggregate(pr, future_lims[0], future_lims[1], nb)
        labels = torch.from_numpy(get_labels_np(vad.numpy(), bin_frames))
        loss = loss_vap(out["logits"], labels)
    if taps is not None:
        taps["logits"], taps["vad_logits"], taps["labels"] = out["logits"], out["vad"], labels
    return {"probs": pr, "vad": vad, "p_now": p_now, "p_future": p_future, "H": H, "loss": loss}


def state_dict_to_torch(sd_np: Dict[str, np.ndarray]) -> SD:
    return {k: torch.from_numpy(np.asarray(v, dtype=np.float32)) for k, v in sd_np.items()}


# --------------------------------------------------------------------------------------------
# VapGPTMono (vap/model.py:271-393)
# --------------------------------------------------------------------------------------------
def encode_va(va: Tensor, sd: SD, va_history: Optional[Tensor] = None) -> Tensor:
    """VapGPTMono.encode_va (model.py:352-357): LN(va_condition(va) [+ va_cond_history(hist)])."""
    v = va @ sd["va_condition.weight"].T + sd["va_condition.bias"]
    if va_history is not None and "va_cond_history.weight" in sd:
        v = v + va_history @ sd["va_cond_history.weight"].T + sd["va_cond_history.bias"]
    return layer_norm(v, sd, "va_cond_ln")


def forward_mono(waveform: Tensor, va: Tensor, sd: SD, va_history: Optional[Tensor] = None,
                 num_heads: int = 4) -> Dict[str, Tensor]:
    """VapGPTMono.forward (model.py:360-393): encoder on one speaker, + encode_va, ar_channel GPT,
    ar GPT (self attention only), vap_head; "vad" is the va input itself."""
    assert waveform.shape[1] == 1, f"audio VAP ENCODER: {waveform.shape} != (B, 1, n_samples)"
    x = encoder(waveform, sd)
    x = x + encode_va(va, sd, va_history)
    for l in range(count_layers(sd, "ar_channel")):
        x = transformer_layer(x, sd, f"ar_channel.layers.{l}", num_heads)
    for l in range(count_layers(sd, "ar")):
        x = transformer_layer(x, sd, f"ar.layers.{l}", num_heads)
    logits = x @ sd["vap_head.weight"].T + sd["vap_head.bias"]
    return {"logits": logits, "vad": va}


def probs_mono(waveform: Tensor, va: Tensor, sd: SD, va_history: Optional[Tensor] = None, num_heads: int = 4,
               now_lims=(0, 1), future_lims=(2, 3), n_bins: int = 4) -> Dict[str, Tensor]:
    """VapGPTMono.probs (model.py:325-350): no labels / loss (unlike VapGPT.probs)."""
    with torch.no_grad():
        out = forward_mono(waveform, va, sd, va_history, num_heads)
        pr = out["logits"].softmax(dim=-1)
        H = (-pr * pr.log2()).sum(dim=-1)
        p_now = probs_next_speaker_aggregate(pr, now_lims[0], now_lims[-1], n_bins)
        p_future = probs_next_speaker_aggregate(pr, future_lims[0], future_lims[1], n_bins)
    return {"probs": pr, "vad": va, "p_now": p_now, "p_future": p_future, "H": H}
