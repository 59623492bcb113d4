"""bench.py's rank launcher on CPU: `--gpus N` with no torchrun environment starts N
fresh ranks itself (the driver may call `python3 bench.py --gpus 8` directly), a
WORLD_SIZE that disagrees with --gpus fails loudly, and a failing rank fails the run.
--dry-run keeps every rank off the GPU (gloo control collectives only) and runs the
per-GPU efficiency arithmetic of the N-rank line on synthetic per-rank times."""
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
    # the per-GPU efficiency fields (solo_times + scaling_fields, the same code the GPU
    # run uses), on synthetic per-rank times: alone 20 ms each, together 20 ms x (1 + r/10)
    sc = line["scaling_check"]
    assert len(sc["per_rank_GiBps"]) == n and len(sc["solo_GiBps"]) == n
    assert sc["solo_GiBps"] == [round((1 << 20) / 0.02 / (1 << 30), 2)] * n
    assert sc["per_gpu_efficiency"] == pytest.approx(1 / (1 + (n - 1) / 10), abs=2e-4)


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


def test_cpu_baseline_threads_follow_the_cgroup_quota(tmp_path):
    """cpu_baseline's core count: the cgroup CPU quota (v2 cpu.max
    or v1 cfs quota / period), capped by the affinity mask; no quota -> the mask."""
    sys.path.insert(0, ROOT)
    import bench

    affinity = len(os.sched_getaffinity(0))
    (tmp_path / "cpu.max").write_text("max 100000\n")
    assert bench.cpu_quota(str(tmp_path)) == (affinity, None, "no cgroup CPU quota: every CPU in the affinity mask")
    (tmp_path / "cpu.max").write_text("200000 100000\n")
    th, q, src = bench.cpu_quota(str(tmp_path))
    assert (th, q) == (min(2, affinity), 2.0) and "cpu.max" in src
    v1 = tmp_path / "v1"
    (v1 / "cpu").mkdir(parents=True)
    (v1 / "cpu" / "cpu.cfs_quota_us").write_text("150000\n")
    (v1 / "cpu" / "cpu.cfs_period_us").write_text("100000\n")
    th, q, src = bench.cpu_quota(str(v1))
    assert (th, q) == (1, 1.5) and "cfs_quota_us" in src
    (v1 / "cpu" / "cpu.cfs_quota_us").write_text("-1\n")
    assert bench.cpu_quota(str(v1))[:2] == (affinity, None)
