"""bench.py --gpus N launches its own N rank processes when no external
launcher set WORLD_SIZE: one process per GPU, started as
children before any GPU call, each told RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT.  Exercised here with the gloo backend on CPU (a
child script that joins the group the launcher describes), plus the refusal
to print a 1-GPU line for --gpus 2 on a box without 2 devices."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = os.path.join(ROOT, "tests", "_launch_child.py")
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _launch(world, argv, timeout=240):
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.launch_ranks(%d, %r, script=%r))" % (ROOT, world, argv, CHILD))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=timeout, env=env)


def test_rank_env():
    e = bench.rank_env({"X": "1"}, 3, 8, 29511)
    assert e["X"] == "1"
    assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"], e["LOCAL_WORLD_SIZE"]) == ("3", "3", "8", "8")
    assert (e["MASTER_ADDR"], e["MASTER_PORT"]) == ("127.0.0.1", "29511")


@pytest.mark.parametrize("world", [2, 4])
def test_launcher_forms_a_world_of_n_ranks(world):
    p = _launch(world, [str(world)])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout            # rank 0's line only
    j = json.loads(lines[0])
    assert j["world_size"] == world and j["sum"] == world * (world + 1) // 2
    assert [r["rank"] for r in j["ranks"]] == list(range(world))
    assert [r["local_rank"] for r in j["ranks"]] == list(range(world))
    assert len({r["pid"] for r in j["ranks"]}) == world     # one process per rank


def test_launcher_fails_when_a_rank_fails():
    """rank 1 exits 3 before joining; rank 0 would wait in the rendezvous
    forever -- the launcher stops it and returns the failing code"""
    p = _launch(2, ["2", "1"])
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    assert "rank 1 exited with 3" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_bench_refuses_more_gpus_than_visible():
    """--gpus 2 with fewer devices: a clear error and a non-zero exit, never a
    1-GPU line labelled as 2"""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("this box has 2 devices")
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 2, (p.returncode, p.stderr[-2000:])
    assert "--gpus 2 needs 2 HIP devices" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_bench_rank_checks_world_against_gpus():
    """a rank whose WORLD_SIZE disagrees with --gpus stops before any GPU work"""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "1"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 2 and "WORLD_SIZE 2 but --gpus 4" in p.stderr, p.stderr[-2000:]
