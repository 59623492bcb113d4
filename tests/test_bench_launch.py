"""bench.py's rank launcher on CPU: `--gpus N` with no torchrun environment starts N
fresh ranks itself (the driver may call `python3 bench.py --gpus 8` directly), a
WORLD_SIZE that disagrees with --gpus fails loudly, and a failing rank fails the run.
--dry-run keeps every rank off the GPU (gloo control collectives only)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def _run(args, env, timeout=150):
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.timeout(180)
@pytest.mark.parametrize("n", [2, 3])
def test_gpus_flag_spawns_ranks(n):
    r = _run(["--gpus", str(n), "--dry-run"], _env())
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints
    line = json.loads(lines[0])
    assert line["n_gpus"] == n
    assert line["pids_distinct"] == n  # n separate processes
    assert line["ranks_ok"] is True


@pytest.mark.timeout(60)
def test_world_size_mismatch_fails_loudly():
    r = _run(["--gpus", "2", "--dry-run"], _env(WORLD_SIZE="4", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0
    assert "WORLD_SIZE=4" in r.stderr


@pytest.mark.timeout(60)
def test_single_gpu_default_needs_no_launcher():
    r = _run(["--dry-run"], _env())
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1


@pytest.mark.timeout(120)
def test_failing_rank_fails_the_run():
    # rank 1 exits before the rendezvous, so rank 0 would wait there forever: the
    # launcher must stop it and return the failing rank's code
    r = _run(["--gpus", "2", "--dry-run"], _env(RSGPU_BENCH_DRY_FAIL_RANK="1"))
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert "rank 1 exited with 3" in r.stderr
