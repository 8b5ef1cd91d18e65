"""The RCCL branch of the multi-GPU step loop (rt_amd/shard.py FrameSteps, backend "nccl"), run on
the one GPU a test box has: a 1-rank nccl process group on device 0.  The gather then goes over
RCCL from the device buffer on torch's stream, and the max-over-ranks all_reduce of the elapsed
time runs on a device tensor — the code path the 8-GPU driver run takes, which the two-rank tests
(gloo, both ranks on device 0, where RCCL refuses) cannot reach.  The assembled frame must equal
the dist=None run bit for bit, in both gather modes ("frame": once at frame end, "step": after
every step)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, math, os, sys
sys.path.insert(0, os.path.join(%(root)r, "gpu-ray_trace-rust_amd"))
sys.path.insert(0, os.path.join(%(root)r, "tests"))
import numpy as np
import torch
import torch.distributed as dist
from conftest import load_scene
from rt_amd import render, shard

torch.cuda.set_device(0)
sc = load_scene("walled", width=256, height=120)
w, h = int(sc.info.width), int(sc.info.height)
tiles = shard.rank_tiles(w, h, 0, 1)
out = {}
with render.Context(sc, device=0) as ctx:
    fs = shard.FrameSteps(ctx, tiles, w, h, 0, 1, shard.stripe_rows(h, 1), 4, 0)
    fs.run(3, 1)
    ref = fs.frame()
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(%(port)d))
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
seen = []  # (collective, tensor device) of every call FrameSteps makes


class Spy:
    ReduceOp = dist.ReduceOp

    def gather(self, t, gather_list=None, dst=0):
        seen.append(("gather", str(t.device)))
        return dist.gather(t, gather_list=gather_list, dst=dst)

    def all_reduce(self, t, op=None):
        seen.append(("all_reduce", str(t.device)))
        return dist.all_reduce(t, op=op)

    def barrier(self):
        return dist.barrier()


try:
    for mode in ("frame", "step"):
        seen.clear()
        with render.Context(sc, device=0) as ctx:
            fs = shard.FrameSteps(ctx, tiles, w, h, 0, 1, shard.stripe_rows(h, 1), 4, 0, dist=Spy(),
                                  backend="nccl", gather=mode)
            r = fs.run(3, 1)
            f = fs.frame()
        out[mode] = {"equal": bool(np.array_equal(f, ref)), "complete": bool((f[..., 3] == 1).all()),
                     "gathers": r["gathers"], "gather_ms_per_gather": r.get("gather_ms_per_gather"),
                     "gather_buffers": [str(b.device) for b in fs.gather], "calls": list(seen)}
finally:
    dist.destroy_process_group()
print("RESULT", json.dumps(out))
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_frame_steps_over_rccl_one_rank(gpu_available):
    code = CHILD % {"root": ROOT, "port": _free_port()}
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-u", "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=240,
                       env=env)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert r.returncode == 0 and line, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(line[0][7:])
    for mode, gathers in (("frame", 1), ("step", 3)):
        m = res[mode]
        assert m["equal"] and m["complete"], m
        assert m["gathers"] == gathers, m
        g = m["gather_ms_per_gather"]
        assert g is not None and g == g and 0 <= g < 1e4, m  # finite CUDA-event time
        assert m["gather_buffers"] == ["cuda:0"], m  # the RCCL gather lands in device memory
        colls = m["calls"]
        # the one warmup step gathers in either mode (it is the last step of its own run)
        assert [c for c in colls if c[0] == "gather"] == [["gather", "cuda:0"]] * (gathers + 1), m
        assert ["all_reduce", "cuda:0"] in colls, m  # max over ranks on a device tensor
