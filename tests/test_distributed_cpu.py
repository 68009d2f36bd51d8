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
        n_classes = 256

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
