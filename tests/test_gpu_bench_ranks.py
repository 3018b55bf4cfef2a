"""GPU check of bench.py's multi-rank path (spawn before any GPU call,
per-rank graph slices, the sharded HIP solve, barrier + max-over-ranks
timing, the JSON line) on the one GPU of the box: --share-gpu puts both ranks
on cuda:0 with gloo collectives (RCCL refuses two ranks on one device). The
driver's SCALE run uses the same code with one GPU per rank over RCCL."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def test_bench_two_ranks_share_gpu():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-gpu", "--steps", "2",
           "--warmup", "1", "--no-cpu", "--no-tracker", "--cold-steps", "0", "--lin-reps", "3",
           "--height", "128", "--width", "128"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2
    assert line["share_gpu"] is True
    assert line["value"] > 0 and line["ms_per_step"] > 0
    assert "world_size=2" in r.stderr  # each rank reports the world it sees
