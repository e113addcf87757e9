"""The --gpus N launcher of bench.py / main.py (viforssms_amd.launch.ensure_world), on CPU: world checks under a
launcher, and a real 2-rank spawn through torchrun (gloo) from a plain `python script --gpus 2`."""
import os
import subprocess
import sys

import pytest

from viforssms_amd import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIST_VARS = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")


def test_world_checks(monkeypatch):
    for v in DIST_VARS:
        monkeypatch.delenv(v, raising=False)
    assert launch.ensure_world(1, "x.py", []) is None           # one rank, no launcher: run here
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert launch.ensure_world(2, "x.py", []) is None           # torchrun started the requested world
    with pytest.raises(SystemExit) as e:
        launch.ensure_world(4, "x.py", [])                      # --gpus disagrees with the launched world
    assert "WORLD_SIZE=2" in str(e.value)
    with pytest.raises(SystemExit):
        launch.ensure_world(0, "x.py", [])


def test_launch_command_rendezvous_on_loopback():
    cmd = launch.rank_launch_cmd(8, "/r/bench.py", ["--gpus", "8", "--steps", "3"], port=29611)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "29611"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"] and cmd[-5] == "/r/bench.py"


def test_plain_python_gpus_2_spawns_two_ranks(tmp_path):
    env = {k: v for k, v in os.environ.items() if k not in DIST_VARS}
    env["PYTHONPATH"] = ROOT
    env["VISSM_DIST_BACKEND"] = "gloo"   # CPU host (an empty HIP_VISIBLE_DEVICES list refuses an RCCL world)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "_launch_probe.py"), "--gpus", "2", str(tmp_path)],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    got = sorted(open(tmp_path / f).read().split() for f in os.listdir(tmp_path))
    assert got == [["0", "2", "2"], ["1", "2", "2"]]


def test_launcher_never_touches_the_gpu_runtime(monkeypatch):
    """The parent that spawns the ranks must not initialise HIP (a GPU-initialised process must not start the
    ranks): ensure_world counts devices from the visibility variables / render nodes, never through torch.cuda."""
    import torch

    def _boom(*a, **k):
        raise AssertionError("the launcher queried the GPU runtime")

    for v in DIST_VARS:
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setattr(torch.cuda, "device_count", _boom)
    monkeypatch.setattr(torch.cuda, "is_available", _boom)
    monkeypatch.setattr(torch._C, "_cuda_getDeviceCount", _boom, raising=False)
    calls = []
    monkeypatch.setattr(launch.subprocess, "call", lambda cmd: calls.append(cmd) or 0)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1")
    assert launch.ensure_world(2, "b.py", ["--gpus", "2"]) == 0
    assert len(calls) == 1 and "--nproc-per-node=2" in calls[0]
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
    with pytest.raises(SystemExit, match="needs 2 visible GPUs"):
        launch.ensure_world(2, "b.py", [])
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")               # an explicitly empty list is zero devices
    assert launch.visible_gpu_count() == 0
    with pytest.raises(SystemExit, match="found 0"):
        launch.ensure_world(2, "b.py", [])
    monkeypatch.setenv("VISSM_DIST_BACKEND", "gloo")            # the one-GPU rehearsal may oversubscribe
    assert launch.ensure_world(2, "b.py", []) == 0
    assert not torch.cuda.is_initialized()
