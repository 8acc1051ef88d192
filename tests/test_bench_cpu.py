"""bench.py's launcher logic (CPU only: nothing here touches a GPU).

`python bench.py --gpus N` must run N ranks itself when no launcher set
WORLD_SIZE, and must refuse a --gpus that disagrees with the launcher's
WORLD_SIZE (the driver runs `torch.distributed.run --nproc-per-node N
bench.py --gpus N`).
"""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_default_is_one_rank_in_process():
    assert bench.resolve_launch(None, {}) == ("self", 1)
    assert bench.resolve_launch(1, {}) == ("self", 1)


def test_gpus_without_launcher_spawns():
    assert bench.resolve_launch(2, {}) == ("spawn", 2)
    assert bench.resolve_launch(8, {"WORLD_SIZE": ""}) == ("spawn", 8)


def test_under_launcher_world_size_rules():
    assert bench.resolve_launch(None, {"WORLD_SIZE": "4"}) == ("self", 4)
    assert bench.resolve_launch(4, {"WORLD_SIZE": "4"}) == ("self", 4)
    assert bench.resolve_launch(1, {"WORLD_SIZE": "1"}) == ("self", 1)
    with pytest.raises(ValueError):
        bench.resolve_launch(2, {"WORLD_SIZE": "4"})
    with pytest.raises(ValueError):
        bench.resolve_launch(0, {})


def test_spawn_command_is_the_driver_form():
    cmd = bench.spawn_command(4, ["--gpus", "4", "--steps", "20"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert "--master-port=29555" in cmd
    assert cmd[-5] == os.path.join(REPO, "bench.py")
    assert cmd[-4:] == ["--gpus", "4", "--steps", "20"]


def test_mismatch_fails_before_any_gpu_work():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "3"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "disagrees with WORLD_SIZE=2" in r.stderr


def test_spawned_ranks_see_world_size(tmp_path, monkeypatch):
    """spawn_ranks runs the launcher; every rank sees WORLD_SIZE == N and
    re-resolves to ("self", N).  A stand-in script takes bench.py's place."""
    probe = tmp_path / "probe.py"
    out = tmp_path / "out"
    probe.write_text(
        "import os, sys\n"
        f"sys.path.insert(0, {REPO!r})\n"
        "import bench\n"
        "how, w = bench.resolve_launch(int(sys.argv[2]), os.environ)\n"
        f"open(os.path.join({str(out)!r} + os.environ['RANK']), 'w').write(f'{{how}} {{w}}')\n")
    monkeypatch.setattr(bench.os.path, "abspath",
                        lambda p, _real=os.path.abspath: str(probe) if p == bench.__file__ else _real(p))
    rc = bench.spawn_ranks(2, ["--gpus", "2"])
    assert rc == 0
    for r in range(2):
        assert open(str(out) + str(r)).read() == "self 2"
