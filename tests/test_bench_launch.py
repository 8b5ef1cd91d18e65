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
    assert launch_cmd(["--gpus", "2", "--frame-abi"], {}) is None  # one process, rt_frame_* over 2 devices


RANKS_CHILD = r"""
import json, os, sys
sys.argv = ["bench.py"]
sys.path.insert(0, %(root)r)
import torch.distributed as dist
import bench
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%(port)d", rank=%(rank)d, world_size=2)
rank = dist.get_rank()
ident = {"rank": rank, "local_rank": rank, "device": rank, "pci_bus_id": "0000:%%02x:00.0" %% (0x11 + rank),
         "uuid": "u%%d" %% rank, "name": "fake", "visible_devices": None}
idents = bench.gather_identities(ident, dist, 2)
print("RESULT " + json.dumps(bench.rank_summary(idents, dist)), flush=True)
dist.destroy_process_group()
"""


def test_rank_identities_gathered_over_two_ranks():
    """The N > 1 line's proof of what ran: every rank's device ordinal and PCI
    location gathered to every rank over a real 2-rank gloo group, the count of distinct devices and
    the group's backend and size — the keys bench.py's N-rank line carries."""
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = [subprocess.Popen([sys.executable, "-c", RANKS_CHILD % {"root": ROOT, "port": port, "rank": r}],
                              cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = [p.communicate(timeout=120) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
    res = [json.loads([ln for ln in o.splitlines() if ln.startswith("RESULT ")][0][7:]) for o, _ in outs]
    assert res[0] == res[1]
    r = res[0]
    assert [i["rank"] for i in r["ranks"]] == [0, 1]
    assert [i["pci_bus_id"] for i in r["ranks"]] == ["0000:11:00.0", "0000:12:00.0"]
    assert r["distinct_devices"] == 2
    assert r["dist"] == {"backend": "gloo", "world_size": 2}
