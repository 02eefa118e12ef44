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


@pytest.mark.parametrize("world", [2, 8])
def test_multi_rank_line_carries_cpu_baseline_and_per_rank_roofline(world):
    """at N > 1 the line keeps the CPU leg (rank 0, after the
    timed region, the other ranks held at a barrier until it ends) and the
    roofline is per GPU -- every rank's kernel time all-gathered, per-rank
    fractions and their minimum; the wall time is the max over ranks."""
    p = _launch(world, [str(world), "-1", "line"], timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    j = json.loads(lines[0])
    assert j["world_size"] == world
    assert j["wall"] == pytest.approx(0.1 * world)
    assert j["kernel_ms"] == [10.0 + r for r in range(world)]
    rows = j["roofline"]["per_rank"]
    assert [r["rank"] for r in rows] == list(range(world))
    assert j["roofline"]["frac_min"] == min(r["frac"] for r in rows) == rows[-1]["frac"]
    assert j["roofline"]["kernel_ms_max"] == 10.0 + world - 1
    cpu = j["cpu_baseline"]
    assert cpu is not None and cpu["value"] > 0 and cpu["cores"] >= 1 and cpu["legs"]
    assert j["e2e"] == {"value": 1.0, "what": "stub"}
    assert j["cpu_ran_on_this_rank"]
    # no rank left the second barrier before rank 0's CPU leg had started
    assert min(j["left_barrier"]) >= j["cpu_started"]


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


def _fake_topology(tmp_path, gpus_minors, cpu_nodes=1, open_minors=None):
    nodes = tmp_path / "nodes"
    dri = tmp_path / "dri"
    nodes.mkdir()
    dri.mkdir()
    k = 0
    for _ in range(cpu_nodes):
        (nodes / str(k)).mkdir()
        (nodes / str(k) / "properties").write_text("cpu_cores_count 64\nsimd_count 0\ndrm_render_minor 0\n")
        k += 1
    for m in gpus_minors:
        (nodes / str(k)).mkdir()
        (nodes / str(k) / "properties").write_text(f"cpu_cores_count 0\nsimd_count 1024\ngfx_target_version 90500\n"
                                                   f"drm_render_minor {m}\n")
        k += 1
    for m in (gpus_minors if open_minors is None else open_minors):
        (dri / f"renderD{m}").write_text("")
    return str(nodes), str(dri)


def test_count_gpus_from_sysfs(tmp_path):
    """the launcher's device count: GPU topology nodes whose render node is
    there to open (a container sees the host's 8 nodes, 2 render nodes), the
    *_VISIBLE_DEVICES caps, and 0 without a KFD tree"""
    nodes, dri = _fake_topology(tmp_path, [128, 136, 144, 152, 160, 168, 176, 184], open_minors=[136, 160])
    assert bench.count_gpus(nodes, dri, env={}) == 2
    assert bench.count_gpus(nodes, dri, env={"HIP_VISIBLE_DEVICES": "0"}) == 1
    assert bench.count_gpus(nodes, dri, env={"ROCR_VISIBLE_DEVICES": "0,1,2"}) == 2
    assert bench.count_gpus(nodes, dri, env={"CUDA_VISIBLE_DEVICES": ""}) == 0
    assert bench.count_gpus(str(tmp_path / "absent"), dri, env={}) == 0


def test_launcher_parent_makes_no_gpu_call(tmp_path):
    """bench.py --gpus N as its own launcher: counting devices and deciding
    (here: refusing, with no devices) never imports torch or loads the HIP
    runtime in the parent -- checked from inside the process at exit"""
    probe = tmp_path / "probe.py"
    probe.write_text(
        "import atexit, sys, runpy\n"
        "def _report():\n"
        "    maps = open('/proc/self/maps').read()\n"
        "    print('PARENT', 'torch' in sys.modules, 'libamdhip64' in maps, 'libtlsrec' in maps, file=sys.stderr)\n"
        "atexit.register(_report)\n"
        f"sys.argv = [{os.path.join(ROOT, 'bench.py')!r}, '--gpus', '2', '--steps', '1']\n"
        f"runpy.run_path({os.path.join(ROOT, 'bench.py')!r}, run_name='__main__')\n")
    env = dict(os.environ, HIP_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, str(probe)], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 2, (p.returncode, p.stderr[-2000:])
    assert "PARENT False False False" in p.stderr, p.stderr[-2000:]


@pytest.mark.gpu
def test_count_gpus_matches_hip():
    """on a GPU box the sysfs count agrees with the HIP runtime's"""
    import torch
    assert bench.count_gpus() == torch.cuda.device_count() >= 1
