#!/usr/bin/env python3
"""Benchmark: Msamples/s (pixels x spp / s) of the MI355X path-tracing hot path on walled.yml.

One step = one launch of the megakernel over this rank's pixels for `--spp-per-step` samples
(the reference's gpu_render_batch, walled.yml: 1000), plus — for N > 1 — the frame-end RCCL
gather of every rank's tile radiance to rank 0.  Inputs (scene, KD tree) are resident in HBM
before the timed region.  N GPUs: one process per GPU (torch.distributed.run), image rows
sharded as 1-row stripes dealt round-robin.  Weak scaling: at N GPUs a step renders N x
spp-per-step samples for every pixel, so each rank keeps the work of the 1-GPU step
(W*H/N pixels x N*spp samples) and the image stays bit-identical to the 1-GPU one (the RNG and
the running mean are keyed on the global pixel and absolute sample index).

Prints ONE JSON line (rank 0) with `roofline` (algorithmic bytes of the trace kernel per
launch / its HIP-event duration vs 8 TB/s HBM) and `cpu_baseline` (the oracle restatement of
the reference CPU renderer on this host, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray_trace-rust_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# Canonical per-event byte sizes of the roofline
BYTES = {"nodes": 8, "leaf_refs": 4, "sphere_tests": 16, "tri_tests": 36, "hits": 32, "mesh_hits": 132}


from rt_amd.shard import STRIPE, max_rank_pixels, rank_tiles  # noqa: E402


def roofline_bytes_per_sample(ctx, width, height, spp=16, device=False):
    """Bytes per sample on every 16th pixel in x and y, 16 spp.  device=False:
    the reference algorithm's work (the §8d algorithmic figure); True: the device path's."""
    tiles = [(x, y, 1, 1) for y in range(0, height, 16) for x in range(0, width, 16)]
    c = ctx.count_work(tiles, 0, spp, device=device)
    total = sum(BYTES[k] * c[k] for k in BYTES)
    trav = sum(BYTES[k] * c[k] for k in ("nodes", "leaf_refs", "sphere_tests", "tri_tests"))
    return total / c["samples"], trav / c["samples"], c


def committed_traffic(scene, samples_per_launch):
    """HBM bytes per launch from the committed rocprofv3 FETCH_SIZE pass of the same workload
    (profiles/*_fetch.json, written by tools/prof_summary.py), or None."""
    import glob

    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_fetch.json"))):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        if d.get("scene") == scene and d.get("samples_per_launch") == samples_per_launch:
            best = (d["hbm_read_bytes_per_launch"], os.path.relpath(p, ROOT))
    return best


# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 2 cycles per SIMD
# (MI355X_MICROARCH.md: SIMD-32, a wave's instruction issues over 2 cycles) at 2.4 GHz
VALU_PEAK_WINST_S = 256 * 4 * 2.4e9 / 2


def committed_valu(scene, samples_per_launch):
    """VALU wave-instructions per launch (and lane utilisation) from the committed rocprofv3 SQ
    passes of the same workload (profiles/*_valu.json, written by tools/prof_summary.py)."""
    import glob

    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_valu.json"))):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        if d.get("scene") == scene and d.get("samples_per_launch") == samples_per_launch:
            best = (d, os.path.relpath(p, ROOT))
    return best


def cpu_baseline(loaded, target_s=10.0, threads=None):
    """The oracle (C++ restatement of render_to_target_cpu) on this host's cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py  # test infrastructure: the CPU baseline leg only

    threads = threads or min(16, os.cpu_count() or 1)
    w, h = int(loaded.info.width), int(loaded.info.height)
    # One oracle call renders a whole frame at `spp` (like render_to_target_cpu: one KD build per
    # frame, then the samples).  spp is sized from the marginal cost of a sample, measured as
    # t(2 spp) - t(1 spp), so that the timed call takes about target_s.
    def timed(n):
        t0 = time.perf_counter()
        oracle_py.render(loaded, [(0, 0, w, h)], 0, n, threads=threads)
        return time.perf_counter() - t0

    t1 = timed(1)
    if t1 < target_s:
        t1 = timed(1)  # the first call also pays one-time loading
    if t1 >= target_s:
        spp, dt = 1, t1
    else:
        per = max(timed(2) - t1, 0.05 * t1)
        spp = max(1, min(256, int(round((target_s - (t1 - per)) / per))))
        dt = timed(spp)
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(w * h * spp / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads,
            "kind": "port", "cpu_model": model, "host_cpus": os.cpu_count(),
            "sample": f"full {w}x{h} frame, {spp} spp in one call (KD build included, as per frame in "
                      f"the reference), oracle/oracle.cpp recursive radiance, {threads} threads, {dt:.1f} s"}


def measured_valu_stream():
    """G wave-instructions/s of a pure full-rate VALU stream (v_fma_f32, distinct operands) from
    the committed tools/valu_rates.hip run (profiles/*_valu_rates.json), or None.  Under a full
    VALU load the chip does not hold 2.4 GHz, so this is the ceiling actually reachable."""
    import glob

    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_valu_rates.json"))):
        try:
            rows = [json.loads(line) for line in open(p) if line.strip()]
        except (OSError, ValueError):
            continue
        for r in rows:
            if r.get("insn") == "v_fma_f32":
                best = (r["G_winst_per_s"], os.path.relpath(p, ROOT))
    return best


def valu_roofline(scene, samples_per_launch, kernel_ms):
    """The bound the kernel actually runs against: VALU instruction issue."""
    c = committed_valu(scene, samples_per_launch)
    if not c:
        return None
    d, src = c
    rate = d["valu_insts_per_launch"] / (kernel_ms * 1e-3)
    out = {"insts_per_launch": d["valu_insts_per_launch"], "achieved_winst_per_s": round(rate / 1e9, 1),
           "peak_winst_per_s": round(VALU_PEAK_WINST_S / 1e9, 1), "unit": "G wave-instructions/s",
           "frac": round(rate / VALU_PEAK_WINST_S, 4), "lane_util": d.get("valu_lane_util"), "source": src}
    m = measured_valu_stream()
    if m:
        out["measured_stream_winst_per_s"] = m[0]
        out["frac_of_measured_stream"] = round(rate / 1e9 / m[0], 4)
        out["measured_stream_source"] = m[1]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="walled")
    ap.add_argument("--spp-per-step", type=int, default=None,
                    help="samples per pixel per launch (default: the scheme's gpu_render_batch)")
    ap.add_argument("--width", type=int, default=None, help="override the scheme's width")
    ap.add_argument("--height", type=int, default=None, help="override the scheme's height")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--as-rank", default=None,
                    help="r/N: time rank r's share of an N-GPU run on this one GPU (no gather); "
                         "a scaling rehearsal, not the contract's multi-process run")
    args = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from rt_amd import render, scheme

    sch = scheme.load_json(os.path.join(ROOT, "tests", "golden", "scenes", args.scene + ".json"))
    loaded = scheme.load(sch, assets_root=os.path.join(ROOT, "assets_pack"), width=args.width, height=args.height)
    w, h = int(loaded.info.width), int(loaded.info.height)
    spp = args.spp_per_step or int(sch["render_info"].get("gpu_render_batch") or 1)
    shard_rank, shard_world = rank, world
    if args.as_rank:
        if world != 1:
            raise SystemExit("--as-rank is a single-process rehearsal")
        shard_rank, shard_world = (int(v) for v in args.as_rank.split("/"))
    tiles = rank_tiles(w, h, shard_rank, shard_world)
    npix = sum(t[2] * t[3] for t in tiles)
    max_npix = max(max_rank_pixels(w, h, world), npix)

    ctx = render.Context(loaded, device=local)
    out = torch.zeros((max_npix, 4), dtype=torch.float32, device=f"cuda:{local}")
    gather = [torch.empty_like(out) for _ in range(world)] if (world > 1 and rank == 0) else None

    def barrier():
        if dist:
            dist.barrier()
        torch.cuda.synchronize()

    sample = 0

    spp_rank = spp * shard_world  # weak scaling: per-rank work is the 1-GPU step's

    def step():
        nonlocal sample
        ctx.render_device(out.data_ptr(), tiles, sample, spp_rank)
        sample += spp_rank
        if dist:
            dist.gather(out, gather_list=gather, dst=0)

    for _ in range(args.warmup):
        step()
    barrier()
    kernel_ms, launch_ms, n_launch = [], [], 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        ls = ctx.launch_stats()
        kernel_ms.append(ls["render_ms"])
        launch_ms.append(ls["trace_ms"])
        n_launch += ls["n_trace_launches"]
    barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # after the timed region: rank 0 reassembles the last gathered frame (rt_amd/shard.py) and
    # checks that every pixel was rendered by some rank (alpha is 1 exactly where written)
    frame_complete = None
    if not args.as_rank and rank == 0:
        from rt_amd import shard

        frame = shard.assemble(gather if dist else [out], w, h, world)
        frame_complete = bool((frame[..., 3] == 1.0).all().item())

    total_samples = (npix if args.as_rank else w * h) * spp_rank * args.steps
    value = total_samples / elapsed / 1e6
    res = {"metric": f"Msamples/s (pixels x spp / s) on {args.scene}.yml",
           "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
           "data": "synthetic-free: the reference's own scene file (tests/golden/scenes), seeded RNG",
           "config": {"workload": f"{args.scene}.yml {w}x{h}, {spp} spp x n_gpus per step (one launch per rank), "
                                  f"kd_tree_depth {int(loaded.info.kd_tree_depth)}",
                      "spp_per_step": spp, "pixels": w * h, "stripes": f"{STRIPE}-row round-robin",
                      "parallelism": f"tiles{world}"}}
    res["frame_complete"] = frame_complete
    res["launch"] = {"trace_launches_per_step": n_launch / args.steps,
                     "samples_per_launch": round(npix * spp_rank * args.steps / max(n_launch, 1))}
    if args.as_rank:
        res["config"]["rehearsal"] = f"rank {shard_rank} of {shard_world}, single GPU, no gather"
        res["scaling"] = None

    if rank == 0 and not args.no_roofline:
        bps, trav_bps, counts = roofline_bytes_per_sample(ctx, w, h)
        dev_bps, _, dev_counts = roofline_bytes_per_sample(ctx, w, h, device=True)
        # per trace launch, like rocprofv3's per-kernel average: a step is n launches of the queue
        # kernel (radiance buffer chunks) plus their in-order folds
        avg_ms = sum(launch_ms) / n_launch
        per_launch = npix * spp_rank * args.steps / n_launch
        achieved = bps * per_launch / (avg_ms * 1e-3) / 1e9
        spheres_only = loaded.desc.n_free_tris == 0 and loaded.desc.n_meshes == 0
        traffic = committed_traffic(args.scene, round(per_launch))
        res["roofline"] = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                           "traffic": traffic[0] if traffic else None,
                           "traffic_unit": "bytes/launch (rocprofv3 FETCH_SIZE x2, gfx950)",
                           "traffic_source": traffic[1] if traffic else None,
                           "algorithmic_bytes_per_launch": round(bps * per_launch),
                           "kernel": f"rtd::queue_kernel<{'false' if spheres_only else 'true'}, {'true' if int(loaded.info.dir_light_samp) else 'false'}>",
                           "kernel_ms_avg": round(avg_ms, 3), "launches_per_step": n_launch / args.steps,
                           "step_device_ms_avg": round(sum(kernel_ms) / len(kernel_ms), 3),
                           "bytes_per_sample": round(bps, 1), "traversal_bytes_per_sample": round(trav_bps, 1),
                           "samples_per_launch": round(per_launch),
                           "counts_per_sample": {k: round(v / counts["samples"], 3) for k, v in counts.items()
                                                 if k != "samples"},
                           "device_bytes_per_sample": round(dev_bps, 1),
                           "device_frac": round(dev_bps * per_launch / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                           "device_counts_per_sample": {k: round(v / dev_counts["samples"], 3)
                                                        for k, v in dev_counts.items() if k != "samples"},
                           "valu": valu_roofline(args.scene, round(per_launch), avg_ms),
                           "note": "achieved/frac price the REFERENCE algorithm's bytes per sample (SURVEY.md "
                                   "§8d, counted by rt_count_work); the device skips provably non-returning "
                                   "KD leaves (closest_small), so frac can exceed 1; device_frac prices the "
                                   "device's own logical reads; traffic is the real HBM read volume"}
    if rank == 0 and world == 1 and not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline(loaded, args.cpu_seconds)
    ctx.close()
    if dist:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
