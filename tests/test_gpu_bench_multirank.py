"""bench.py's own multi-rank path, run as the driver launches it: two processes
under torch.distributed.run, each rank rendering its stripes with rt_render_device_async, one
gather per step (rt_amd/shard.py FrameSteps), the max-over-ranks timing and rank 0's frame
assembly.  On one GPU both ranks share device 0, so the gather goes over gloo from host copies
(--dist-backend gloo; RCCL refuses two ranks on one device); on an 8-GPU node the same code path
gathers device buffers over RCCL.  The assembled frame must be complete and equal the 1-rank
frame bit for bit, for the strong (fixed-frame) headline and for the weak run."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench(tmp_path, tag, world, extra):
    dump = str(tmp_path / f"{tag}.npy")
    args = ["bench.py", "--gpus", str(world), "--steps", "2", "--warmup", "1", "--no-cpu", "--no-roofline",
            "--no-configs", "--dump-frame", dump] + extra
    if world > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args + \
              ["--dist-backend", "gloo", "--same-device"]
    else:
        cmd = [sys.executable] + args
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, r.stdout  # one JSON line, from rank 0 only
    return json.loads(line[0]), np.load(dump)


@pytest.mark.parametrize("scene,spp", [("walled", 8), ("biplane", 2)])
def test_bench_two_ranks_equal_one(gpu_available, tmp_path, scene, spp):
    one, f1 = _bench(tmp_path, "one", 1, ["--scene", scene, "--spp-per-step", str(spp)])
    two, f2 = _bench(tmp_path, "two", 2, ["--scene", scene, "--spp-per-step", str(spp)])
    assert one["frame_complete"] and two["frame_complete"]
    assert two["n_gpus"] == 2 and two["scaling"] == "strong"
    assert two["config"]["dist_backend"] == "gloo" and "weak" in two and "gather_ms_per_step" in two
    # strong: both runs render [0, 3 spp) of every pixel (1 warmup + 2 timed steps)
    assert np.array_equal(f1, f2)
    assert (f2[..., 3] == 1.0).all()
    # weak headline: each rank renders 2 x spp per step; the frame equals 1 rank at 2 x spp
    weak, fw = _bench(tmp_path, "weak", 2, ["--scene", scene, "--spp-per-step", str(spp), "--weak"])
    one2, f12 = _bench(tmp_path, "one2", 1, ["--scene", scene, "--spp-per-step", str(2 * spp)])
    assert weak["scaling"] == "weak" and "strong" in weak
    assert np.array_equal(fw, f12)
