"""bench.py --gpus N (the driver's contract): without a launcher it starts torchrun as a child
process with one rank per GPU (never exec'ing itself), and it refuses a world size that does
not match --gpus, so an N-GPU line can never silently measure one GPU."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_launcher_command_line():
    cmd = bench.launcher_cmd(["--gpus", "4", "--steps", "7"], 4, 29517)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd and "--master-port=29517" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "7"]
    assert os.path.samefile(cmd[-5], os.path.join(REPO, "bench.py"))


def test_world_size_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "--gpus 4 but WORLD_SIZE=2" in r.stderr


@pytest.mark.parametrize("n", [1])
def test_free_port(n):
    p = bench.free_port()
    assert 1024 < p < 65536
