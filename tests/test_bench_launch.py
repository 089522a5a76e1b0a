"""bench.py's launcher (CPU, no GPU work): `bench.py --gpus N` run directly
starts N ranks itself, and a launcher-provided WORLD_SIZE must match --gpus."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env,
                          capture_output=True, text=True, timeout=120)


def test_gpus_n_spawns_n_ranks():
    r = _run(["--gpus", "3", "--dry-run"])
    assert r.returncode == 0, r.stderr
    lines = [json.loads(s) for s in r.stdout.splitlines() if s.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1, 2]
    assert sorted(x["local_rank"] for x in lines) == [0, 1, 2]
    assert all(x["world"] == 3 and x["master"] == "127.0.0.1" for x in lines)


def test_single_gpu_runs_in_process():
    r = _run(["--gpus", "1", "--dry-run"])
    assert r.returncode == 0, r.stderr
    lines = [json.loads(s) for s in r.stdout.splitlines() if s.startswith("{")]
    assert lines == [{"rank": 0, "local_rank": 0, "world": 1, "master": lines[0]["master"]}]


def test_world_size_mismatch_fails():
    r = _run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE 4" in r.stderr
