"""bench.py's launch contract on a CPU-only host (no GPU): ``--gpus N``
spawns N ranks (one process per GPU) and reports n_gpus = N; under a launcher
a WORLD_SIZE that differs from --gpus is refused. ``--dry-run`` replaces the
per-rank HIP compute with no-op ops over gloo, so only the orchestration
(spawn, collectives, max-over-ranks timing, JSON line) is exercised."""
import json
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _run(args, env_extra=None):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env,
                          capture_output=True, text=True, timeout=240)


def test_gpus_2_spawns_two_ranks():
    r = _run(["--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1", "--cold-steps", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1  # rank 0 prints exactly one JSON line
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["dry_run"] is True
    assert d["config"]["keyframes"] == 64  # weak scaling: 32 KFs per rank
    assert "world_size=2" in r.stderr


def test_world_size_mismatch_is_refused():
    r = _run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "4"})
    assert r.returncode == 2
    assert "refusing" in r.stderr
