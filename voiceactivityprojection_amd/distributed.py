"""Data-parallel inference across the GPUs of a node (one process per GPU, RCCL over xGMI).

The VAP forward has no cross-clip dependency (every op is per batch element), so clips shard as
contiguous slices of the global batch with replicated weights and NO collective on the data path;
the only exchange is one gather of the per-frame outputs to rank 0 (north_star: "a single RCCL
gather over xGMI for the output probabilities").  The reference has no inference parallelism
(training only: Lightning DDP, vap/train.py:237); this module is new.

Works with any torch.distributed backend: "nccl" (= RCCL on ROCm) on the GPU node, "gloo" in the
CPU tests (tests/test_distributed_cpu.py).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .utils import frame_lengths

COMPACT_KEYS = ("p_now", "p_future", "vad", "H")


def shard_range(global_batch: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [start, stop) slice of the global batch for `rank` (sizes differ by at most 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, extra = divmod(global_batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_outputs(out: Dict[str, torch.Tensor], keys: Sequence[str] = COMPACT_KEYS, dst: int = 0,
                   group=None) -> Optional[Dict[str, torch.Tensor]]:
    """Gather per-rank output tensors (batch-first) to `dst`, concatenated in rank order.

    Ranks may hold different batch sizes (shard_range): sizes are exchanged first (one tiny
    all_gather), then every key is padded to the max local batch for the gather and trimmed on
    `dst`.  Returns the concatenated dict on `dst`, None elsewhere.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    ref = out[keys[0]]
    n_local = torch.tensor([ref.shape[0]], dtype=torch.int64, device=ref.device)
    sizes = [torch.zeros_like(n_local) for _ in range(world)]
    dist.all_gather(sizes, n_local, group=group)
    sizes = [int(s.item()) for s in sizes]
    nmax = max(sizes)
    res: Dict[str, torch.Tensor] = {}
    for k in keys:
        t = out[k].contiguous()
        if t.shape[0] < nmax:
            pad = torch.zeros((nmax - t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            t = torch.cat([t, pad], 0)
        bufs: Optional[List[torch.Tensor]] = [torch.empty_like(t) for _ in range(world)] if rank == dst else None
        dist.gather(t, bufs, dst=dst, group=group)
        if rank == dst:
            res[k] = torch.cat([b[:s] for b, s in zip(bufs, sizes)], 0)
    return res if rank == dst else None


def empty_probs(n_samples: int, device, n_classes: int = 256, horizon_frames: int = 100) -> Dict[str, torch.Tensor]:
    """Zero-clip ``probs()`` outputs for ``n_samples`` per channel: the shapes a 0-row batch would have
    (probs (0, T, 256), vad / p_now / p_future (0, T, 2), H (0, T), loss (0, T - horizon))."""
    T = frame_lengths(n_samples)[-1]
    z = lambda *shape: torch.zeros(shape, dtype=torch.float32, device=device)  # noqa: E731
    return {"probs": z(0, T, n_classes), "vad": z(0, T, 2), "p_now": z(0, T, 2), "p_future": z(0, T, 2),
            "H": z(0, T), "loss": z(0, max(T - horizon_frames, 0))}


def probs_sharded(model, waveform_global: torch.Tensor, rank: int, world: int, device,
                  keys: Sequence[str] = COMPACT_KEYS, group=None):
    """Run ``model.probs`` on this rank's slice of a global batch and gather to rank 0.

    A rank whose slice is empty (global batch < world) skips the engine (which rejects a batch of
    0) and still joins the gather with zero-row outputs of the right trailing shapes, so no rank is
    left waiting in the collective."""
    s, e = shard_range(waveform_global.shape[0], rank, world)
    if e > s:
        out = model.probs(waveform_global[s:e].to(device))
    else:
        out = empty_probs(waveform_global.shape[-1], device, model.objective.n_classes,
                          int(round(model.horizon_time * model.frame_hz)))
    return gather_outputs(out, keys, dst=0, group=group)
