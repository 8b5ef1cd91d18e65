"""a380 at 1 spp per call (bench config 2's launch shape) through FrameSteps after a long warmup
(the first ~100 launches of a process run ~25% slower); env knobs of the launch pipeline
(GPU_MAX_HW_QUEUES, RT_DEBUG_LAUNCH slots / grid_div) are read per process."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (sets GPU_MAX_HW_QUEUES before HIP starts)
from rt_amd import render  # noqa: E402
from rt_amd.shard import FrameSteps, rank_tiles  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "a380"
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 1
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
tag = os.environ.get("TAG", "")
_, loaded = bench.load(scene)
w, h = int(loaded.info.width), int(loaded.info.height)
for c in range(int(os.environ.get("CTXS", "1"))):  # fresh contexts in turn (new slot streams)
    ctx = render.Context(loaded, device=0)
    fs = FrameSteps(ctx, rank_tiles(w, h, 0, 1, 8), w, h, 0, 1, 8, spp, 0)
    vals = []
    for k in range(3):
        r = fs.run(steps, 8 if k or c else steps)
        vals.append(round(w * h * spp * steps / r["elapsed_s"] / 1e6, 1))
    print("RES", tag, "ctx", c, scene, spp, vals, round(r["launch"]["trace_ms"] / r["launch"]["n_timed_launches"], 2),
          flush=True)
    del fs
    ctx.close()
