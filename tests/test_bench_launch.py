"""bench.py --gpus N (BASELINE.json metric "1/2/4/8 MI355X"): without
WORLD_SIZE the bench starts N ranks itself (torch.distributed.run on
127.0.0.1) before touching the GPU; with WORLD_SIZE set it must equal N.
CPU only: the launched ranks stop before any GPU work (--ranks-check)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def test_launch_plan():
    assert bench.launch_plan(1, {}) == "inproc"
    assert bench.launch_plan(2, {}) == "spawn"
    assert bench.launch_plan(8, {}) == "spawn"
    assert bench.launch_plan(2, {"WORLD_SIZE": "2"}) == "inproc"
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}) == "inproc"
    assert bench.launch_plan(8, {"WORLD_SIZE": "1"}).startswith("error")
    assert bench.launch_plan(1, {"WORLD_SIZE": "4"}).startswith("error")


def test_rank_command():
    cmd = bench.rank_command(4, ["--gpus", "4", "--steps", "3"], 29500)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-port=29500" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, capture_output=True, text=True,
                          timeout=240, env=env, cwd=str(ROOT))


def test_gpus_2_starts_two_ranks():
    r = _run(["--gpus", "2", "--ranks-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert sorted(l["rank"] for l in lines) == [0, 1]
    assert all(l["world"] == 2 and l["gpus"] == 2 for l in lines)


def test_world_mismatch_exits_nonzero():
    r = _run(["--gpus", "8", "--ranks-check"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr


@pytest.mark.parametrize("gpus", [1])
def test_single_gpu_runs_in_process(gpus):
    r = _run(["--gpus", str(gpus), "--ranks-check"])
    assert r.returncode == 0
    assert json.loads(r.stdout.strip().splitlines()[-1]) == {"rank": 0, "world": 1, "gpus": 1}
