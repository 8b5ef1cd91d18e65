#!/usr/bin/env python3
"""Benchmark: Msamples/s (pixels x spp / s) of the MI355X path-tracing hot path on walled.yml.

One step = one batch (the reference's gpu_render_batch, walled.yml: 1000 spp) over this rank's
pixels: rt_render_device_async, which overlaps step i + 1's trace with step i's drain tail
(draw_scene.rs:30-44's batches are independent sample ranges; only their running-mean folds are
ordered), plus — for N > 1 — the frame-end RCCL gather of every rank's tile radiance to rank 0,
on torch's stream behind the step's fold.  Inputs (scene, KD tree) are resident in HBM before the
timed region.  N GPUs: one process per GPU (torch.distributed.run), image rows dealt to ranks as
1-row stripes.  Default weak scaling: at N GPUs a step renders N x spp samples for every pixel,
so each rank keeps the 1-GPU step's work (W*H/N pixels x N*spp samples).  --strong keeps the
frame fixed (W*H*spp per step over all ranks; BASELINE config 5 is spaceship_r1 4096^2 at 1000
spp = `--scene spaceship_r1 --width 4096 --height 4096 --spp-per-step 25 --strong --steps 40`).
Either way the image is bit-identical to the 1-GPU one (the RNG and the running mean are keyed
on the global pixel and the absolute sample index).

Prints ONE JSON line (rank 0).  `roofline` names the measured limiter of the trace kernel:
VALU issue (SQ_INSTS_VALU per launch over the launch's HIP-event duration, against 256 CUs x
4 SIMDs x one wave64 instruction per 2 cycles at 2.4 GHz) unless HBM traffic (FETCH_SIZE x 2)
is the larger fraction.  Counter values come from the committed rocprofv3 passes
(profiles/*_counters.json) of the SAME kernel build — keyed on a hash of the library's device
code, so a kernel change without a re-profile prints null instead of a stale figure.  SURVEY.md
§8d's algorithmic bytes of the reference's traversal are reported apart (`reference_work`):
the device skips most of that work exactly, so they are not a roofline.
`cpu_baseline` is the oracle restatement of the reference CPU renderer on all host cores.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray_trace-rust_amd"))
# rt_amd raises HIP's hardware queues per process (GPU_MAX_HW_QUEUES, before HIP starts) so that
# the pipeline slots' streams overlap instead of sharing queues (launch pipeline)
import rt_amd  # noqa: E402,F401

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md §L2: ~34.5 TB/s chip-wide
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 2 cycles per SIMD
# (MI355X_MICROARCH.md: SIMD-32, a wave's instruction issues over 2 cycles) at 2.4 GHz
VALU_PEAK_WINST_S = 256 * 4 * 2.4e9 / 2
# Canonical per-event byte sizes of the reference algorithm's work
BYTES = {"nodes": 8, "leaf_refs": 4, "sphere_tests": 16, "tri_tests": 36, "hits": 32, "mesh_hits": 132}


from rt_amd.shard import max_rank_pixels, rank_tiles, stripe_rows  # noqa: E402


def reference_bytes_per_sample(ctx, width, height, spp=16, device=False):
    """Bytes per sample on every 16th pixel in x and y, 16 spp.  device=False:
    the reference algorithm's work; True: the device path's."""
    tiles = [(x, y, 1, 1) for y in range(0, height, 16) for x in range(0, width, 16)]
    c = ctx.count_work(tiles, 0, spp, device=device)
    total = sum(BYTES[k] * c[k] for k in BYTES)
    return total / c["samples"], c


def committed_counters(build_id, scene, samples_per_launch):
    """The rocprofv3 counters of this kernel build on this workload (tools/prof_summary.py)."""
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_counters.json"))):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        if (d.get("build_id") == build_id and d.get("scene") == scene
                and d.get("samples_per_launch") == samples_per_launch):
            best = (d, os.path.relpath(p, ROOT))
    return best


def measured_valu_stream():
    """G wave-instructions/s of a pure v_fma_f32 stream (tools/valu_rates.hip, committed): under a
    full VALU load the chip does not hold 2.4 GHz, so this is the rate actually reachable."""
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_valu_rates.json"))):
        try:
            for line in open(p):
                r = json.loads(line) if line.strip() else {}
                if r.get("insn") == "v_fma_f32":
                    return r["G_winst_per_s"], os.path.relpath(p, ROOT)
        except (OSError, ValueError):
            continue
    return None


def roofline(scene, per_launch, kernel_ms, build_id, kernel):
    """Measured fractions of the trace kernel's ceilings; bound = the largest."""
    out = {"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": None,
           "kernel": kernel, "kernel_ms_avg": round(kernel_ms, 3), "samples_per_launch": round(per_launch),
           "build_id": build_id, "counters_source": None}
    c = committed_counters(build_id, scene, round(per_launch))
    if not c:
        out["note"] = "no committed rocprofv3 counters for this kernel build and workload: re-profile"
        return out
    d, src = c
    sec = kernel_ms * 1e-3
    out["counters_source"] = src
    fr = {}
    if d.get("valu_insts_per_launch"):
        rate = d["valu_insts_per_launch"] / sec
        v = {"achieved": round(rate / 1e9, 1), "peak": round(VALU_PEAK_WINST_S / 1e9, 1),
             "unit": "G VALU wave-instructions/s", "frac": round(rate / VALU_PEAK_WINST_S, 4),
             "insts_per_launch": d["valu_insts_per_launch"], "lane_util": d.get("valu_lane_util")}
        m = measured_valu_stream()
        if m:
            v["measured_fma_stream"] = m[0]
            v["frac_of_measured_stream"] = round(rate / 1e9 / m[0], 4)
        out["valu"] = v
        fr["valu"] = v
    if d.get("hbm_read_bytes_per_launch"):
        t = d["hbm_read_bytes_per_launch"]
        out["traffic"] = t
        h = {"achieved": round(t / sec / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(t / sec / 1e9 / HBM_PEAK_GBS, 4), "bytes_per_launch": t,
             "note": "rocprofv3 FETCH_SIZE x2 (gfx950 correction, MI355X_MICROARCH.md), own pass"}
        out["hbm"] = h
        fr["hbm"] = h
    if d.get("td_busy_frac"):
        # the vector-memory pipeline: fraction of the kernel's cycles the per-CU texture-data unit
        # (the return path of every global / scratch load) is busy; the mesh kernels' limiter
        v = {"achieved": d["td_busy_frac"], "peak": 1.0, "unit": "fraction of cycles TD busy",
             "frac": d["td_busy_frac"], "ta_busy_frac": d.get("ta_busy_frac"),
             "note": "rocprofv3 TD_TD_BUSY_sum / 256 CUs over GRBM_GUI_ACTIVE / 8 XCDs, own pass"}
        out["vmem"] = v
        fr["vmem"] = v
    if d.get("l2_bytes_per_launch"):
        b = d["l2_bytes_per_launch"]
        out["l2"] = {"achieved": round(b / sec / 1e9, 1), "peak": L2_PEAK_GBS, "unit": "GB/s",
                     "frac": round(b / sec / 1e9 / L2_PEAK_GBS, 4), "hit_rate": d.get("l2_hit_rate"),
                     "note": "(TCC_HIT + TCC_MISS) x 128 B, own pass"}
    for k in ("wait_any_frac", "issue_frac", "issue_stall_frac"):
        if k in d:
            out.setdefault("wave_cycles", {})[k] = d[k]
    if fr:
        b = max(fr, key=lambda k: fr[k]["frac"])
        out.update(bound=b, achieved=fr[b]["achieved"], peak=fr[b]["peak"], unit=fr[b]["unit"],
                   frac=fr[b]["frac"])
        if out["frac"] > 1.0:  # a counter from another workload or a broken timer: refuse it
            out.update(bound=None, achieved=None, frac=None, note=f"refused: frac {out['frac']} > 1")
    return out


def cpu_baseline(loaded, target_s=15.0, threads=None):
    """The oracle (C++ restatement of render_to_target_cpu, recursive radiance) on every host core
    (the reference's rayon par_iter_mut uses all of them, draw_scene.rs:73).  The KD build and
    scene setup are timed apart (an oracle call with 0 samples), as SURVEY.md §8d asks."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py  # test infrastructure: the CPU baseline leg only

    threads = threads or os.cpu_count() or 1
    w, h = int(loaded.info.width), int(loaded.info.height)
    full = [(0, 0, w, h)]

    def timed(n):
        t0 = time.perf_counter()
        oracle_py.render(loaded, full, 0, n, threads=threads)
        return time.perf_counter() - t0

    timed(0)  # one-time loading
    t_build = min(timed(0), timed(0))
    t1 = timed(1) - t_build
    spp = max(1, min(1024, int(target_s / max(t1, 1e-3))))
    dt = timed(spp) - t_build
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(w * h * spp / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads,
            "kind": "port", "cpu_model": model, "host_cpus": os.cpu_count(), "kd_build_s": round(t_build, 3),
            "sample": f"full {w}x{h} frame, {spp} spp in one call on {threads} threads ({dt:.1f} s after "
                      f"the KD build); oracle/oracle.cpp recursive radiance"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="walled")
    ap.add_argument("--spp-per-step", type=int, default=None,
                    help="samples per pixel per step (default: the scheme's gpu_render_batch)")
    ap.add_argument("--width", type=int, default=None, help="override the scheme's width")
    ap.add_argument("--height", type=int, default=None, help="override the scheme's height")
    ap.add_argument("--strong", action="store_true", help="fixed frame: N ranks split W*H*spp per step")
    ap.add_argument("--sync", action="store_true", help="synchronous steps (rt_render_device), for A/B")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=None)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--stripe", type=int, default=None,
                    help="rows per stripe (default: rt_amd.shard.stripe_rows, equal stripe counts per rank)")
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

    from rt_amd import abi, render, scheme

    sch = scheme.load_json(os.path.join(ROOT, "tests", "golden", "scenes", args.scene + ".json"))
    loaded = scheme.load(sch, assets_root=os.path.join(ROOT, "assets_pack"), width=args.width, height=args.height)
    w, h = int(loaded.info.width), int(loaded.info.height)
    spp = args.spp_per_step or int(sch["render_info"].get("gpu_render_batch") or 1)
    shard_rank, shard_world = rank, world
    if args.as_rank:
        if world != 1:
            raise SystemExit("--as-rank is a single-process rehearsal")
        shard_rank, shard_world = (int(v) for v in args.as_rank.split("/"))
    stripe = args.stripe or stripe_rows(h, shard_world)
    tiles = rank_tiles(w, h, shard_rank, shard_world, stripe)
    npix = sum(t[2] * t[3] for t in tiles)
    max_npix = max(max_rank_pixels(w, h, world, stripe), npix)

    ctx = render.Context(loaded, device=local)
    out = torch.zeros((max_npix, 4), dtype=torch.float32, device=f"cuda:{local}")
    gather = [torch.empty_like(out) for _ in range(world)] if (world > 1 and rank == 0) else None
    stream = torch.cuda.current_stream().cuda_stream

    def barrier():
        if dist:
            dist.barrier()
        torch.cuda.synchronize()

    sample = 0
    spp_rank = spp if args.strong else spp * shard_world  # weak: per-rank work is the 1-GPU step's
    gather_ev = []

    def step():
        nonlocal sample
        if args.sync:
            ctx.render_device(out.data_ptr(), tiles, sample, spp_rank)
        else:
            ctx.render_device_async(out.data_ptr(), tiles, sample, spp_rank, stream=stream)
        sample += spp_rank
        if dist:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            dist.gather(out, gather_list=gather, dst=0)
            e1.record()
            gather_ev.append((e0, e1))

    for _ in range(args.warmup):
        step()
    ctx.synchronize()
    barrier()
    gather_ev.clear()
    sync_stats = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        if args.sync:
            sync_stats.append(ctx.launch_stats())  # each synchronous call is its own window
    ctx.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    # every trace launch of the timed steps (HIP events on their streams)
    ls = ctx.launch_stats() if not args.sync else {
        k: sum(s[k] for s in sync_stats) for k in ("render_ms", "trace_ms", "n_trace_launches")}
    if dist:
        t = torch.tensor([elapsed], device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # after the timed region: rank 0 reassembles the last gathered frame (rt_amd/shard.py) and
    # checks that every pixel was rendered by some rank (alpha is 1 exactly where written)
    frame_complete = None
    if not args.as_rank and rank == 0:
        from rt_amd import shard

        frame = shard.assemble(gather if dist else [out], w, h, world, stripe)
        frame_complete = bool((frame[..., 3] == 1.0).all().item())

    # every rank renders its pixels x spp_rank per step (weak: spp x N, strong: spp)
    total_samples = (npix if args.as_rank else w * h) * spp_rank * args.steps
    value = total_samples / elapsed / 1e6
    n_launch = ls["n_trace_launches"]
    per_launch = npix * spp_rank * args.steps / max(n_launch, 1)
    kernel_ms = ls["trace_ms"] / max(n_launch, 1)
    spheres_only = loaded.desc.n_free_tris == 0 and loaded.desc.n_meshes == 0
    kernel = (f"rtd::queue_kernel<{'false' if spheres_only else 'true'}, "
              f"{'true' if int(loaded.info.dir_light_samp) else 'false'}>")
    res = {"metric": f"Msamples/s (pixels x spp / s) on {args.scene}.yml",
           "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
           "higher_is_better": True, "scaling": "strong" if args.strong else "weak", "vs_baseline": None,
           "dtype": "f32",
           "data": "synthetic-free: the reference's own scene file (tests/golden/scenes), seeded RNG",
           "config": {"workload": f"{args.scene}.yml {w}x{h}, {spp} spp per step"
                                  f"{'' if args.strong else ' x n_gpus'} (one queue launch per rank and step), "
                                  f"kd_tree_depth {int(loaded.info.kd_tree_depth)}",
                      "spp_per_step": spp, "pixels": w * h, "stripes": f"{stripe}-row round-robin",
                      "parallelism": f"tiles{world}", "dispatch": "sync" if args.sync else "async"}}
    res["frame_complete"] = frame_complete
    res["launch"] = {"trace_launches_per_step": n_launch / args.steps, "samples_per_launch": round(per_launch),
                     "trace_ms_per_launch": round(kernel_ms, 3),
                     "device_window_ms": round(ls["render_ms"], 3)}
    if gather_ev:
        res["gather_ms_per_step"] = round(sum(a.elapsed_time(b) for a, b in gather_ev) / len(gather_ev), 3)
    if args.as_rank:
        res["config"]["rehearsal"] = f"rank {shard_rank} of {shard_world}, single GPU, no gather"
        res["scaling"] = None

    if rank == 0 and not args.no_roofline:
        res["roofline"] = roofline(args.scene, per_launch, kernel_ms, abi.kernel_build_id(), kernel)
        bps, counts = reference_bytes_per_sample(ctx, w, h)
        dev_bps, dev_counts = reference_bytes_per_sample(ctx, w, h, device=True)
        res["reference_work"] = {
            "bytes_per_sample": round(bps, 1), "bytes_per_launch": round(bps * per_launch),
            "GB_s": round(bps * per_launch / (kernel_ms * 1e-3) / 1e9, 1),
            "counts_per_sample": {k: round(v / counts["samples"], 3) for k, v in counts.items() if k != "samples"},
            "device_bytes_per_sample": round(dev_bps, 1),
            "device_counts_per_sample": {k: round(v / dev_counts["samples"], 3)
                                         for k, v in dev_counts.items() if k != "samples"},
            "note": "SURVEY.md §8d canonical bytes of the REFERENCE algorithm's work (rt_count_work), priced "
                    "per launch over the launch's duration: not a roofline, the device skips most of this "
                    "work exactly (closest_small, DESIGN.md §5)"}
    if rank == 0 and world == 1 and not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline(loaded, args.cpu_seconds, args.cpu_threads)
    ctx.close()
    if dist:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
