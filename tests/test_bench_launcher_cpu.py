"""bench.py --gpus N launcher (one process per GPU) exercised on CPU in its gloo
--dry-run mode: N ranks start, see a world of N with distinct local ranks, and exactly one JSON
line is printed (by rank 0)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]  # gloo logs its own lines
    return lines


@pytest.mark.parametrize("n", [1, 2])
def test_launcher_dry_run(n):
    lines = _run("--gpus", str(n), "--dry-run", "--steps", "3", "--warmup", "1")
    assert len(lines) == 1, lines
    out = json.loads(lines[0])
    assert out["n_gpus"] == n
    assert out["process_group"]["world_size"] == n
    assert sorted(out["process_group"]["local_ranks"]) == list(range(n))
    assert out["steps"] == 3 and out["warmup"] == 1


def test_launcher_propagates_failure():
    """A rank that dies must not leave the others waiting in a collective: the parent stops them
    and exits non-zero."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
    env["ECO_BENCH_DRY_FAIL_RANK"] = "1"
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-run"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
