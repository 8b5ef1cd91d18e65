"""bench.py --gpus N without a launcher starts its own N ranks: the child
command it builds is pinned here on the CPU.  It is torch.distributed.run on one node with the
ranks on 127.0.0.1 and the same arguments, started as a child process (never an exec of the
parent), and nothing is launched when this process already is a rank, runs one GPU, or is bench's
own single-process child.  tests/test_gpu_bench_multirank.py runs it end to end on the GPU."""
import json
import os
import subprocess
import sys

from conftest import ROOT


def launch_cmd(argv, env):
    code = ("import json, sys; sys.argv = ['bench.py']; import bench; "
            "print(json.dumps(bench.self_launch_cmd(%r, %r, 29123)))" % (argv, env))
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_child_command_line():
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    cmd = launch_cmd(argv, {})
    assert cmd[1:] == ["-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "8",
                       "--master-addr", "127.0.0.1", "--master-port", "29123",
                       os.path.join(ROOT, "bench.py")] + argv
    assert os.path.basename(cmd[0]).startswith("python")


def test_gpus_equals_form_and_extra_flags():
    argv = ["--gpus=2", "--dist-backend", "gloo", "--same-device", "--frame-digest"]
    cmd = launch_cmd(argv, {})
    assert cmd[cmd.index("--nproc-per-node") + 1] == "2"
    assert cmd[-len(argv):] == argv


def test_no_launch_when_not_needed():
    assert launch_cmd(["--gpus", "8"], {"WORLD_SIZE": "8"}) is None  # already a rank (driver's torchrun)
    assert launch_cmd(["--gpus", "1"], {}) is None
    assert launch_cmd([], {}) is None
    assert launch_cmd(["--gpus", "4", "--config-only", "a380"], {}) is None
    assert launch_cmd(["--gpus", "4", "--as-rank", "0/4"], {}) is None
