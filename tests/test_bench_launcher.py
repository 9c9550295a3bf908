"""bench.py's multi-rank launcher (no GPU): `--gpus N` starts N rank processes with distinct
RANK / LOCAL_RANK, the same WORLD_SIZE and rendezvous, before any torch/HIP call; a WORLD_SIZE
set by an outer launcher must agree with --gpus."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=120)


def test_launcher_starts_n_ranks():
    r = _run(["--gpus", "4", "--launch-dry-run"])
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.strip()]
    assert sorted(x["rank"] for x in lines) == [0, 1, 2, 3]
    assert sorted(x["local_rank"] for x in lines) == [0, 1, 2, 3]
    assert {x["world"] for x in lines} == {4}
    assert len({tuple(x["master"]) for x in lines}) == 1 and lines[0]["master"][0] == "127.0.0.1"


def test_single_gpu_runs_in_process():
    r = _run(["--launch-dry-run"])
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.strip()]
    assert lines == [{"rank": 0, "local_rank": 0, "world": 1, "master": [None, None]}]


def test_outer_launcher_world_must_match():
    r = _run(["--gpus", "2", "--launch-dry-run"], {"WORLD_SIZE": "8", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=8" in r.stderr
    r = _run(["--gpus", "2", "--launch-dry-run"], {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1"})
    assert r.returncode == 0 and json.loads(r.stdout)["rank"] == 1


def test_failing_rank_fails_the_launch():
    # without a GPU (this container) every rank fails at torch.cuda.set_device: the launcher
    # returns the failing rank's status and says which rank it was
    import torch
    if torch.cuda.is_available():
        import pytest
        pytest.skip("needs a host without a GPU")
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0 and "bench.py: rank" in r.stderr
