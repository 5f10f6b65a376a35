"""bench.py's rank launcher (CPU): `--gpus N` without torch.distributed.run
around the process starts one child, torch.distributed.run with N ranks of the
same command, and forwards rank 0's JSON line and the child's exit status; a
WORLD_SIZE that differs from --gpus is refused before anything else runs.
`--dry-run` makes every rank report its rank and world and exit before any
GPU use, so the launch itself is checked here without a GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


@pytest.mark.parametrize("gpus", [2, 3])
def test_gpus_n_launches_n_ranks(gpus):
    p = subprocess.run([sys.executable, BENCH, "--gpus", str(gpus), "--dry-run"], capture_output=True, text=True,
                       timeout=240, env=_env())
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout  # rank 0's line only; the launcher's chatter goes to stderr
    rec = json.loads(lines[0])
    assert rec == {"dry_run": True, "rank": 0, "world": gpus, "gpus": gpus}
    assert "torch.distributed.run" in p.stderr and f"--nproc-per-node={gpus}" in p.stderr


def test_world_size_mismatch_refused():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], capture_output=True, text=True,
                       timeout=120, env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"))
    assert p.returncode == 2
    assert "WORLD_SIZE=3 but --gpus 2" in p.stderr
    assert p.stdout.strip() == ""


def test_one_gpu_and_inside_a_launcher_run_in_process():
    sys.path.insert(0, ROOT)
    import bench

    class A:
        gpus = 1
    old = os.environ.pop("WORLD_SIZE", None)
    try:
        assert bench.launch_ranks(A) is None  # N = 1: this process is the rank
        os.environ["WORLD_SIZE"] = "1"
        assert bench.launch_ranks(A) is None
        A.gpus = 4
        os.environ["WORLD_SIZE"] = "4"
        assert bench.launch_ranks(A) is None  # already one of 4 ranks
    finally:
        os.environ.pop("WORLD_SIZE", None)
        if old is not None:
            os.environ["WORLD_SIZE"] = old
    cmd = bench.rank_launch_cmd(8, ["--gpus", "8", "--steps", "5"], 29555)
    assert cmd[1:] == ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8", "--master-addr",
                       "127.0.0.1", "--master-port=29555", BENCH, "--gpus", "8", "--steps", "5"]
