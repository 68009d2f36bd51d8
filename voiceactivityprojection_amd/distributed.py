"""Data-parallel inference across the GPUs of a node (one process per GPU, RCCL over xGMI).

The VAP forward has no cross-clip dependency (every op is per batch element), so clips shard as
contiguous slices of the global batch with replicated weights and NO collective on the data path;
the only exchange is ONE gather of the outputs to rank 0 (north_star: "a single RCCL gather over
xGMI for the output probabilities").  The reference has no inference parallelism (training only:
Lightning DDP, vap/train.py:237); this module is new.

Every rank writes its ``probs()`` outputs straight into one packed buffer (:class:`PackedOutputs`,
key-major: all clips' probs, then vad, p_now, p_future, H, loss), so a step ships one contiguous
buffer per rank in one ``gather`` and rank 0 unpacks it.  Shard sizes follow from
:func:`shard_range`, so no size exchange is needed; uneven shards are padded to the largest.

Works with any torch.distributed backend: "nccl" (= RCCL on ROCm) on the GPU node, "gloo" in the
CPU tests (tests/test_distributed_cpu.py).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .utils import frame_lengths

OUTPUT_KEYS = ("probs", "vad", "p_now", "p_future", "H", "loss")
COMPACT_KEYS = ("p_now", "p_future", "vad", "H")


def shard_range(global_batch: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [start, stop) slice of the global batch for `rank` (sizes differ by at most 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, extra = divmod(global_batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard_sizes(global_batch: int, world: int) -> List[int]:
    return [e - s for s, e in (shard_range(global_batch, r, world) for r in range(world))]


def output_shapes(frames: int, n_classes: int = 256, horizon_frames: int = 100) -> Dict[str, Tuple[int, ...]]:
    """Per-clip shapes of ``VapGPT.probs`` outputs (vap/model.py:180-225) for T = ``frames``."""
    return {"probs": (frames, n_classes), "vad": (frames, 2), "p_now": (frames, 2), "p_future": (frames, 2),
            "H": (frames,), "loss": (max(frames - horizon_frames, 0),)}


class PackedOutputs:
    """One contiguous fp32 buffer holding ``capacity`` clips of the selected outputs, key-major:
    ``views(n)`` gives per-key contiguous (n, ...) tensors (the first n clips of each key's region)
    that ``VapGPT.probs(..., out=...)`` writes in place; ``flat`` is what the gather ships."""

    def __init__(self, capacity: int, frames: int, device, keys: Sequence[str] = OUTPUT_KEYS,
                 n_classes: int = 256, horizon_frames: int = 100, flat: Optional[torch.Tensor] = None):
        shapes = output_shapes(frames, n_classes, horizon_frames)
        self.keys = tuple(keys)
        self.capacity = int(capacity)
        self.shapes = {k: shapes[k] for k in self.keys}
        self.per_clip = {k: _numel(self.shapes[k]) for k in self.keys}
        self.numel = self.capacity * sum(self.per_clip.values())
        self.flat = flat if flat is not None else torch.empty(self.numel, dtype=torch.float32, device=device)
        assert self.flat.numel() == self.numel and self.flat.dtype == torch.float32

    def views(self, n: Optional[int] = None, flat: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
        n = self.capacity if n is None else n
        assert 0 <= n <= self.capacity
        buf = self.flat if flat is None else flat
        out, off = {}, 0
        for k in self.keys:
            size = self.capacity * self.per_clip[k]
            out[k] = buf[off: off + n * self.per_clip[k]].view(n, *self.shapes[k])
            off += size
        return out


def _numel(shape) -> int:
    n = 1
    for s in shape:
        n *= s
    return n


def gather_packed(packed: PackedOutputs, dst: int = 0, group=None, recv: Optional[List[torch.Tensor]] = None,
                  async_op: bool = False):
    """ONE ``dist.gather`` of the packed buffer to ``dst``.  Returns (work, recv buffers on dst)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if rank == dst and recv is None:
        recv = [torch.empty_like(packed.flat) for _ in range(world)]
    work = dist.gather(packed.flat, recv if rank == dst else None, dst=dst, group=group, async_op=async_op)
    return work, (recv if rank == dst else None)


def unpack_gathered(packed: PackedOutputs, recv: Sequence[torch.Tensor], sizes: Sequence[int]) -> Dict[str, torch.Tensor]:
    """Concatenate every rank's first ``sizes[r]`` clips per key, in rank order."""
    per_rank = [packed.views(n, flat=buf) for buf, n in zip(recv, sizes)]
    return {k: torch.cat([v[k] for v in per_rank], 0) for k in packed.keys}


def gather_outputs(out: Dict[str, torch.Tensor], keys: Sequence[str] = COMPACT_KEYS, dst: int = 0,
                   group=None, sizes: Optional[Sequence[int]] = None) -> Optional[Dict[str, torch.Tensor]]:
    """Gather per-rank output tensors (batch-first) to ``dst`` in one collective, concatenated in rank
    order.  ``sizes`` = every rank's clip count (default: exchanged with one tiny all_gather)."""
    world = dist.get_world_size(group)
    ref = out[keys[0]]
    if sizes is None:
        n_local = torch.tensor([ref.shape[0]], dtype=torch.int64, device=ref.device)
        got = [torch.zeros_like(n_local) for _ in range(world)]
        dist.all_gather(got, n_local, group=group)
        sizes = [int(s.item()) for s in got]
    T = ref.shape[1]
    n_classes = out["probs"].shape[-1] if "probs" in out else 256
    horizon = T - out["loss"].shape[1] if "loss" in out else 100
    packed = PackedOutputs(max(sizes), T, ref.device, keys, n_classes, horizon)
    packed.flat.zero_()
    views = packed.views(ref.shape[0])
    for k in keys:
        views[k].copy_(out[k])
    _, recv = gather_packed(packed, dst=dst, group=group)
    return unpack_gathered(packed, recv, sizes) if recv is not None else None


def empty_probs(n_samples: int, device, n_classes: int = 256, horizon_frames: int = 100) -> Dict[str, torch.Tensor]:
    """Zero-clip ``probs()`` outputs for ``n_samples`` per channel: the shapes a 0-row batch would have
    (probs (0, T, 256), vad / p_now / p_future (0, T, 2), H (0, T), loss (0, T - horizon))."""
    T = frame_lengths(n_samples)[-1]
    return {k: torch.zeros((0,) + s, dtype=torch.float32, device=device)
            for k, s in output_shapes(T, n_classes, horizon_frames).items()}


def probs_sharded(model, waveform_global: torch.Tensor, rank: int, world: int, device,
                  keys: Sequence[str] = OUTPUT_KEYS, group=None):
    """Run ``model.probs`` on this rank's slice of a global batch, writing into one packed buffer,
    and gather it to rank 0 in ONE collective.  Returns the global outputs on rank 0, None elsewhere.

    A rank whose slice is empty (global batch < world) skips the engine (which rejects a batch of
    0) and still joins the gather, so no rank is left waiting in the collective.  The model's
    hand-off check (``model.synchronize()``) runs before the results are used."""
    gb = waveform_global.shape[0]
    sizes = shard_sizes(gb, world)
    s, e = shard_range(gb, rank, world)
    T = frame_lengths(waveform_global.shape[-1])[-1]
    horizon = int(model.objective.horizon)  # sum of the truncated bin frames, as probs() sizes `loss`
    packed = PackedOutputs(max(sizes), T, device, keys, model.objective.n_classes, horizon)
    packed.flat.zero_()
    if e > s:
        views = packed.views(e - s)
        model.probs(waveform_global[s:e].to(device), out=views)
    sync = getattr(model, "synchronize", None)
    if sync is not None and e > s:
        sync()
    _, recv = gather_packed(packed, dst=0, group=group)
    return unpack_gathered(packed, recv, sizes) if recv is not None else None
