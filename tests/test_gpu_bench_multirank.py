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


def _bench(tmp_path, tag, world, extra, launcher=True, steps=2, warmup=1, dump=True, timeout=240, env_extra=None):
    dump_path = str(tmp_path / f"{tag}.npy")
    args = ["bench.py", "--gpus", str(world), "--steps", str(steps), "--warmup", str(warmup), "--no-cpu",
            "--no-roofline", "--no-configs"] + (["--dump-frame", dump_path] if dump else []) + extra
    if world > 1:
        args += ["--dist-backend", "gloo", "--same-device"]
    if world > 1 and launcher:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
    else:  # one GPU, or N ranks started by bench.py itself (no launcher: the driver's plain command)
        cmd = [sys.executable] + args
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", **(env_extra or {}))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, r.stdout  # one JSON line, from rank 0 only
    return json.loads(line[0]), (np.load(dump_path) if dump else None)


@pytest.mark.parametrize("scene,spp", [("walled", 8), ("biplane", 2)])
def test_bench_two_ranks_equal_one(gpu_available, tmp_path, scene, spp):
    one, f1 = _bench(tmp_path, "one", 1, ["--scene", scene, "--spp-per-step", str(spp)])
    two, f2 = _bench(tmp_path, "two", 2, ["--scene", scene, "--spp-per-step", str(spp)])
    assert one["frame_complete"] and two["frame_complete"]
    assert two["n_gpus"] == 2 and two["scaling"] == "strong"
    assert two["config"]["dist_backend"] == "gloo" and "weak" in two and "gather_ms_per_step" in two
    # what ran: both ranks' devices (here both device 0), the group's backend and size
    assert [i["rank"] for i in two["ranks"]] == [0, 1] and [i["device"] for i in two["ranks"]] == [0, 0]
    assert two["distinct_devices"] == 1 and two["dist"] == {"backend": "gloo", "world_size": 2}
    assert one["ranks"][0]["pci_bus_id"] == two["ranks"][0]["pci_bus_id"]
    # rank 0's C-ABI leg over the ranks' devices (rt_frame_*, two contexts on device 0)
    assert two["frame_abi"]["n_parts"] == 2 and two["frame_abi"]["devices"] == [0, 0], two["frame_abi"]
    assert two["frame_abi"]["value"] > 0
    # strong: both runs render [0, 3 spp) of every pixel (1 warmup + 2 timed steps)
    assert np.array_equal(f1, f2)
    assert (f2[..., 3] == 1.0).all()
    # weak headline: each rank renders 2 x spp per step; the frame equals 1 rank at 2 x spp
    weak, fw = _bench(tmp_path, "weak", 2, ["--scene", scene, "--spp-per-step", str(spp), "--weak"])
    one2, f12 = _bench(tmp_path, "one2", 1, ["--scene", scene, "--spp-per-step", str(2 * spp)])
    assert weak["scaling"] == "weak" and "strong" in weak
    assert np.array_equal(fw, f12)


def test_bench_starts_its_own_ranks(gpu_available, tmp_path):
    """`python bench.py --gpus 2` with no launcher (the driver's plain command line) starts the two
    ranks itself (torch.distributed.run as a child) and prints rank 0's one line: n_gpus 2, the
    frame complete and equal to one rank's bit for bit."""
    one, f1 = _bench(tmp_path, "one", 1, ["--scene", "walled", "--spp-per-step", "8"])
    two, f2 = _bench(tmp_path, "self", 2, ["--scene", "walled", "--spp-per-step", "8"], launcher=False)
    assert two["n_gpus"] == 2 and two["frame_complete"] and two["launcher"] == "bench.py"
    assert np.array_equal(f1, f2)


def test_config5_eight_ranks_on_one_gpu(gpu_available, tmp_path):
    """BASELINE config 5's exact split — spaceship_r1 at 4096 x 4096 over 8 ranks (8-row stripes, 64
    per rank), the 8-way gather and rank 0's assembly — as bench.py runs it, with every rank on
    device 0 (gloo), 1 spp per step, 2 steps: the strong headline (gather at frame end), the
    per-step gather and the weak run (8 spp per rank-step) each equal the 1-rank frame of the same
    samples bit for bit (sha256 of the assembled frames)."""
    common = ["--scene", "spaceship_r1", "--width", "4096", "--height", "4096", "--frame-digest"]
    q4 = {"GPU_MAX_HW_QUEUES": "4"}  # eight processes share one GPU's hardware queues
    eight, _ = _bench(tmp_path, "eight", 8, common + ["--spp-per-step", "1"], launcher=False, warmup=0,
                      dump=False, timeout=600, env_extra=q4)
    one, _ = _bench(tmp_path, "one1", 1, common + ["--spp-per-step", "1"], warmup=0, dump=False)
    one8, _ = _bench(tmp_path, "one8", 1, common + ["--spp-per-step", "8"], warmup=0, dump=False)
    assert eight["n_gpus"] == 8 and eight["frame_complete"] and eight["config"]["stripes"] == "8-row round-robin"
    assert eight["gather"]["gathers"] == 1  # the frame-end gather: once per frame
    assert eight["frame_sha256"] == one["frame_sha256"]
    assert eight["gather_step"]["frame_sha256"] == one["frame_sha256"]
    assert eight["weak"]["spp_per_rank_step"] == 8
    assert eight["weak"]["frame_sha256"] == one8["frame_sha256"]
    # rank 0's C-ABI leg: the same split by rt_frame_* (8 contexts on the ranks' device 0)
    assert eight["frame_abi"]["n_parts"] == 8 and eight["frame_abi"]["stripe_rows"] == 8
    assert eight["frame_abi"]["frame_sha256"] == one["frame_sha256"]


def _bench_frame_abi(tmp_path, devices, extra, env_extra=None, steps=2, warmup=1):
    args = [sys.executable, "bench.py", "--frame-abi", "--gpus", str(len(devices)), "--frame-devices",
            ",".join(str(d) for d in devices), "--steps", str(steps), "--warmup", str(warmup), "--no-cpu",
            "--no-roofline", "--no-configs", "--frame-digest"] + extra
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", **(env_extra or {}))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run(args, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, r.stdout
    return json.loads(line[0])


@pytest.mark.parametrize("staging", [False, True])
def test_bench_frame_abi_equals_one(gpu_available, tmp_path, staging):
    """`bench.py --frame-abi --gpus 2` (one process, rt_frame_* with two contexts, here both on
    device 0; with RT_DEBUG_FRAME_STAGING=1 the second one gathered through the remote-device
    branch) renders the 1-rank frame bit for bit (sha256), reports the contexts' devices and the
    gather's peer-copy and placement times."""
    one, _ = _bench(tmp_path, "one", 1, ["--scene", "walled", "--spp-per-step", "8", "--frame-digest"], dump=False)
    env = {"RT_DEBUG_FRAME_STAGING": "1"} if staging else None
    fa = _bench_frame_abi(tmp_path, [0, 0], ["--scene", "walled", "--spp-per-step", "8"], env_extra=env)
    assert fa["n_gpus"] == 2 and fa["scaling"] == "strong" and fa["config"]["parallelism"] == "frame_abi2"
    assert fa["frame_complete"] and fa["frame_sha256"] == one["frame_sha256"]
    r = fa["frame_abi"]
    assert r["n_parts"] == 2 and r["devices"] == [0, 0] and fa["distinct_devices"] == 1
    assert r["n_peer_copies"] == (2 if staging else 0)  # one per gather: after the warm-up and the timed steps
    assert r["place_ms"] >= 0.0 and r["value"] == fa["value"]
