"""Multi-rank data-parallel path on CPU (gloo, world_size 2): sharding + the single output gather
give the same per-clip results as one process.  Compute on CPU via the oracle (checker only)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from voiceactivityprojection_amd.distributed import empty_probs, gather_outputs, probs_sharded, shard_range


def test_shard_range_covers_batch():
    for gb in (1, 5, 64, 512, 513):
        for world in (1, 2, 3, 8):
            spans = [shard_range(gb, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == gb
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_q):
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (repo, os.path.join(repo, "oracle")):
        sys.path.insert(0, p)
    import vap_oracle as O
    from voiceactivityprojection_amd.weights import synthetic_state_dict, synthetic_waveform

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    sd = O.state_dict_to_torch(synthetic_state_dict(seed=0))
    gb, n = 3, 36000  # odd global batch: shards of 2 and 1
    s, e = shard_range(gb, rank, world)
    w = torch.from_numpy(np.stack([synthetic_waveform(400 + i, n) for i in range(s, e)]))
    out = O.probs(w, sd)
    res = gather_outputs(out, ("p_now", "p_future", "vad", "H"), dst=0)
    if rank == 0:
        out_q.put({k: v.numpy() for k, v in res.items()})
    dist.destroy_process_group()


@pytest.mark.slow
def test_two_rank_gather_equals_single_process():
    import vap_oracle as O
    from voiceactivityprojection_amd.weights import synthetic_state_dict, synthetic_waveform

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sd = O.state_dict_to_torch(synthetic_state_dict(seed=0))
    w = torch.from_numpy(np.stack([synthetic_waveform(400 + i, 36000) for i in range(3)]))
    ref = O.probs(w, sd)
    for k in ("p_now", "p_future", "vad", "H"):
        np.testing.assert_allclose(got[k], ref[k].numpy(), atol=1e-5, rtol=1e-5)  # CPU thread-count noise


class _OracleModel:
    """CPU stand-in for VapGPT (the oracle is the checker here, not the product)."""

    sample_rate, frame_hz, horizon_time = 16000, 50, 2.0

    class objective:
        n_classes, horizon = 256, 100

    def __init__(self, sd):
        self.sd = sd
        self.calls = 0

    def probs(self, w, out=None):
        import vap_oracle as O

        self.calls += 1
        assert w.shape[0] > 0, "the engine rejects an empty batch"
        res = O.probs(w, self.sd)
        for k, v in (out or {}).items():
            v.copy_(res[k])
        return res


def _empty_shard_worker(rank, world, port, out_q):
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (repo, os.path.join(repo, "oracle")):
        sys.path.insert(0, p)
    import vap_oracle as O
    from voiceactivityprojection_amd.weights import synthetic_state_dict, synthetic_waveform

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    m = _OracleModel(O.state_dict_to_torch(synthetic_state_dict(seed=0)))
    w = torch.from_numpy(np.stack([synthetic_waveform(500, 36000)]))  # global batch 1 < world 3
    res = probs_sharded(m, w, rank, world, "cpu")
    out_q.put((rank, m.calls, None if res is None else {k: v.numpy() for k, v in res.items()}))
    dist.destroy_process_group()


def test_empty_probs_shapes():
    e = empty_probs(320000, "cpu")
    assert e["probs"].shape == (0, 1000, 256) and e["H"].shape == (0, 1000) and e["loss"].shape == (0, 900)
    assert e["vad"].shape == e["p_now"].shape == e["p_future"].shape == (0, 1000, 2)


@pytest.mark.slow
def test_empty_shards_join_the_gather():
    """Global batch 1 over 3 ranks: ranks 1 and 2 hold no clip, skip the engine and still take part
    in the gather (no hang); rank 0 gets exactly the one clip's outputs."""
    import vap_oracle as O
    from voiceactivityprojection_amd.weights import synthetic_state_dict, synthetic_waveform

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_empty_shard_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = dict((r, (c, o)) for r, c, o in (q.get(timeout=300) for _ in range(3)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [got[r][0] for r in range(3)] == [1, 0, 0]
    assert got[1][1] is None and got[2][1] is None
    sd = O.state_dict_to_torch(synthetic_state_dict(seed=0))
    ref = O.probs(torch.from_numpy(np.stack([synthetic_waveform(500, 36000)])), sd)
    for k in ("probs", "p_now", "p_future", "vad", "H", "loss"):
        assert got[0][1][k].shape == tuple(ref[k].shape)
        np.testing.assert_allclose(got[0][1][k], ref[k].numpy(), atol=1e-5, rtol=1e-5)


class _ShapeModel:
    """probs() with the engine's strict `out` checks (VapGPT.probs: loss is (B, T - objective.horizon)) and
    the reference objective for any bin_times; writes clip-tagged values."""

    sample_rate, frame_hz = 16000, 50

    def __init__(self, bin_times):
        from voiceactivityprojection_amd.objective import ObjectiveVAP

        self.objective = ObjectiveVAP(bin_times=bin_times, frame_hz=50)
        self.horizon_time = self.objective.horizon_time

    def probs(self, w, out):
        from voiceactivityprojection_amd.utils import frame_lengths

        B, T = w.shape[0], frame_lengths(w.shape[-1])[-1]
        shapes = {"probs": (B, T, 256), "vad": (B, T, 2), "p_now": (B, T, 2), "p_future": (B, T, 2), "H": (B, T),
                  "loss": (B, T - self.objective.horizon)}
        for k, v in out.items():
            if tuple(v.shape) != shapes[k]:
                raise ValueError(f"out[{k!r}] must be {shapes[k]}, got {tuple(v.shape)}")
            v.copy_(w[:, :1, :1].reshape(B, *([1] * (v.dim() - 1))).expand_as(v))
        return out


def test_probs_sharded_non_whole_frame_bins():
    """bin_times that are not whole frames (0.15 s, 0.35 s at 50 Hz: 7 and 17 frames, horizon 94, while
    round(horizon_time * frame_hz) = 95): the packed `loss` region must follow objective.horizon."""
    port = _free_port()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        m = _ShapeModel([0.15, 0.35, 0.6, 0.8])
        assert m.objective.horizon == 94 and round(m.horizon_time * m.frame_hz) == 95
        w = torch.arange(3, dtype=torch.float32).view(3, 1, 1).expand(3, 2, 48000).contiguous()
        res = probs_sharded(m, w, 0, 1, "cpu")
        T = 150
        assert res["loss"].shape == (3, T - 94) and res["probs"].shape == (3, T, 256)
        assert torch.equal(res["H"][:, 0], torch.arange(3, dtype=torch.float32))
    finally:
        dist.destroy_process_group()
