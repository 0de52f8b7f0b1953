"""bench.py's world-size contract (CPU: nothing here touches a GPU).

`python bench.py --gpus N` without a launcher must start its N ranks itself
(torch.distributed.run as a child, before any GPU call); under a launcher
WORLD_SIZE must equal --gpus, else the run fails loudly instead of silently
measuring one GPU.
"""
import os
import subprocess
import sys
import types

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  pylint: disable=g-import-not-at-top


def _args(gpus):
  return types.SimpleNamespace(gpus=gpus)


def test_no_launcher_one_gpu_runs_in_process():
  assert bench.check_world(_args(1), {}) is None


def test_no_launcher_many_gpus_spawns():
  assert bench.check_world(_args(8), {}) == "spawn"
  assert bench.check_world(_args(2), {"RANK": "0"}) == "spawn"


def test_launcher_world_must_match_gpus():
  assert bench.check_world(_args(4), {"WORLD_SIZE": "4"}) is None
  with pytest.raises(SystemExit, match="WORLD_SIZE=2 from the launcher but --gpus 8"):
    bench.check_world(_args(8), {"WORLD_SIZE": "2"})
  with pytest.raises(SystemExit):
    bench.check_world(_args(1), {"WORLD_SIZE": "8"})


def test_launcher_cmd_starts_n_ranks_of_this_script():
  cmd = bench.launcher_cmd(["--gpus", "4", "--steps", "3"], 4, 29511)
  assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
  assert cmd[cmd.index("--nproc-per-node") + 1] == "4"
  assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
  assert cmd[cmd.index("--master-port") + 1] == "29511"
  assert os.path.samefile(cmd[cmd.index("--master-port") + 2], os.path.join(ROOT, "bench.py"))
  assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]


def test_mismatch_fails_before_any_gpu_work():
  env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
  r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"], env=env,
                     capture_output=True, text=True, timeout=300)
  assert r.returncode != 0
  assert "WORLD_SIZE=2 from the launcher but --gpus 8" in r.stderr
