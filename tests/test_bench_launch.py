"""bench.py's multi-rank launch: `python bench.py --gpus N`
without a launcher starts N ranks through one torch.distributed.run child,
relays rank 0's JSON line and checks its n_gpus.  Exercised on the CPU with
--dry-run (gloo ranks, no GPU)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                          timeout=timeout, cwd=ROOT)


@pytest.mark.parametrize("n", [1, 2])
def test_gpus_n_launches_n_ranks(n):
    p = _run(["--gpus", str(n), "--dry-run", "--steps", "3", "--warmup", "1"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout  # exactly one JSON line on stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["steps"] == 3 and out["dry_run"]


def test_world_size_mismatch_fails():
    # a rank whose WORLD_SIZE differs from --gpus refuses to run
    p = _run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert p.returncode != 0
