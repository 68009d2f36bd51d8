"""bench.py's multi-GPU contract, rehearsed on CPU: ``--gpus N`` without a torchrun environment starts N
ranks itself (torchrun as a child process), every rank's outputs travel to rank 0 in ONE gather per
step (packed buffer), the timing is max-over-ranks, and rank 0 prints one JSON line.  ``--stub``
swaps the GPU engine for a step that writes rank-tagged outputs and the RCCL backend for gloo."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO, env=env,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.slow
def test_launcher_spawns_ranks_and_gathers_once():
    p = _run(["--gpus", "2", "--stub", "--batch", "3", "--seconds", "2.5", "--steps", "3", "--warmup", "1"])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 6 and d["config"]["parallelism"] == "dp2"
    assert d["value"] > 0 and d["steps"] == 3 and d["scaling"] == "weak"
    g = d["gather"]
    assert g["calls_per_step"] == 1 and g["verified"] is True
    # every rank's first and last clip was recomputed alone on rank 0 and matched bit for bit
    assert sorted((c["rank"], c["clip"]) for c in g["clips_checked"]) == [(0, 0), (0, 2), (1, 3), (1, 5)]
    assert all(c["bit_identical"] for c in g["clips_checked"])
    assert g["keys"] == ["probs", "vad", "p_now", "p_future", "H", "loss"]
    T = 125  # 2.5 s -> 125 frames; per clip: probs T*256 + 3 * T*2 + H T + loss T-100
    assert g["bytes_per_rank"] == 3 * 4 * (T * 256 + 3 * T * 2 + T + (T - 100))


def test_world_size_must_match_gpus():
    p = _run(["--gpus", "2", "--stub", "--batch", "1", "--seconds", "2.5", "--steps", "1"],
             env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "one rank per GPU" in (p.stderr + p.stdout)


@pytest.mark.slow
def test_exact_check_catches_a_wrong_shard_offset():
    """A rank that computes the wrong clips (its shard shifted by one clip) passes a finiteness check but
    not the exact per-rank recomputation: the bench reports verified=false and exits non-zero."""
    p = _run(["--gpus", "2", "--stub", "--stub-wrong-offset", "--batch", "3", "--seconds", "2.5", "--steps", "2",
              "--warmup", "1"])
    assert p.returncode != 0, (p.returncode, p.stderr[-2000:])  # rank 0 exits 3; torchrun reports 1
    d = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][0])
    g = d["gather"]
    assert g["verified"] is False
    bad = {(c["rank"], c["clip"]) for c in g["clips_checked"] if not c["bit_identical"]}
    assert bad == {(1, 3), (1, 5)}


def _run_stream(args, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    return subprocess.run([sys.executable, os.path.join(REPO, "tools", "bench_stream.py")] + args, cwd=REPO, env=env,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.slow
def test_stream_launcher_shards_streams_and_gathers_each_push():
    """C5 across ranks (tools/bench_stream.py --gpus N): rank r owns streams [r*S, (r+1)*S); every push
    ships its new-hop outputs to rank 0 in ONE gather; the last push's regions hold exactly each rank's
    streams (rank-tagged stub outputs), first and last stream of every rank checked."""
    p = _run_stream(["--gpus", "2", "--stub", "--streams-per-gpu", "3", "--steps", "3", "--warmup", "2"])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["streams"] == 6 and d["streams_per_gpu"] == 3 and d["value"] > 0
    g = d["gather"]
    assert g["calls_per_step"] == 1 and g["verified"] is True
    assert g["bytes_per_rank"] == 3 * 4 * 50 * (256 + 3 * 2 + 1)
    assert sorted((c["rank"], c["stream"]) for c in g["clips_checked"]) == [(0, 0), (0, 2), (1, 3), (1, 5)]


@pytest.mark.slow
def test_stream_launcher_catches_a_wrong_shard_offset():
    p = _run_stream(["--gpus", "2", "--stub", "--stub-wrong-offset", "--streams-per-gpu", "3", "--steps", "2",
                     "--warmup", "1"])
    assert p.returncode != 0
    d = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][0])
    assert d["gather"]["verified"] is False
    assert {(c["rank"], c["stream"]) for c in d["gather"]["clips_checked"] if not c["bit_identical"]} == {(1, 3), (1, 5)}
