"""CPU tests of bench.py's `--gpus N` launcher (bench.py launch_cmd / launch /
main): the driver's N-GPU scaling run goes through it.  The reference
launches one process per GPU from its `cli` (gsplat/distributed.py:304-360);
here the parent starts `torch.distributed.run` as a child process and must
not touch the GPU itself (no device query, no exec)."""

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_launch_cmd_shape():
    sys.path.insert(0, ROOT)
    import bench
    cmd = bench.launch_cmd(8, ["--gpus", "8", "--steps", "5"], 29512)
    assert cmd[0] == sys.executable
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    i = cmd.index("--master-addr")
    assert cmd[i + 1] == "127.0.0.1"
    j = cmd.index("--master-port")
    assert cmd[j + 1] == "29512"
    script = os.path.abspath(os.path.join(ROOT, "bench.py"))
    k = cmd.index(script)
    assert cmd[k + 1:] == ["--gpus", "8", "--steps", "5"]
    assert k > j  # the script and its flags come after the launcher's own


# The parent process: bench.main() with --gpus N and no torchrun environment.
# subprocess.run is replaced by a recorder returning exit code 3, and every
# torch.cuda entry point that would initialise the GPU raises.
_PARENT = r"""
import os, sys, subprocess
sys.path.insert(0, {root!r})
import torch
def _boom(*a, **k):
    raise RuntimeError("parent touched the GPU")
for name in ("is_available", "init", "set_device", "synchronize", "current_device",
             "get_device_properties", "mem_get_info"):
    setattr(torch.cuda, name, _boom)
seen = {{}}
class R:  # CompletedProcess stand-in
    returncode = 3
def fake_run(cmd, env=None, **kw):
    seen["cmd"], seen["env"] = cmd, env
    return R()
subprocess.run = fake_run
import bench
sys.argv = ["bench.py", "--gpus", "4", "--steps", "2", "--warmup", "1"]
try:
    bench.main()
except SystemExit as e:
    code = e.code
assert "torch.distributed.run" in seen["cmd"], seen
assert "--nproc-per-node=4" in seen["cmd"], seen["cmd"]
assert seen["env"].get("HSA_ENABLE_IPC_MODE_LEGACY") == "0"
assert "gsplat_hip" not in sys.modules, "the parent imported the HIP backend"
assert not any(m.startswith("oracle.cpu_step") for m in sys.modules), "CPU pool started in parent"
print("EXIT", code)
"""


def test_parent_launches_child_and_propagates_exit_code():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "-c", _PARENT.format(root=ROOT)], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "EXIT 3" in r.stdout, r.stdout


@pytest.mark.parametrize("world,gpus", [("2", "1"), ("1", "2")])
def test_world_size_must_match_gpus(world, gpus):
    # inside a torchrun environment --gpus must equal WORLD_SIZE (bench.py main)
    env = dict(os.environ, WORLD_SIZE=world, RANK="0", LOCAL_RANK="0")
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.argv = ['bench.py', '--gpus', %r]; bench.main()" % (ROOT, gpus))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0
    assert f"--gpus {gpus} but WORLD_SIZE={world}" in r.stderr, r.stderr[-2000:]
