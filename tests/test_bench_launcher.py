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
    assert g["keys"] == ["probs", "vad", "p_now", "p_future", "H", "loss"]
    T = 125  # 2.5 s -> 125 frames; per clip: probs T*256 + 3 * T*2 + H T + loss T-100
    assert g["bytes_per_rank"] == 3 * 4 * (T * 256 + 3 * T * 2 + T + (T - 100))


def test_world_size_must_match_gpus():
    p = _run(["--gpus", "2", "--stub", "--batch", "1", "--seconds", "2.5", "--steps", "1"],
             env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "one rank per GPU" in (p.stderr + p.stdout)
