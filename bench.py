#!/usr/bin/env python3
"""Benchmark: Msamples/s (pixels x spp / s) of the MI355X path-tracing hot path on walled.yml.

One step = one batch (the reference's gpu_render_batch, walled.yml: 1000 spp) over this rank's
pixels: rt_render_device_async, which overlaps step i + 1's trace with step i's drain tail
(draw_scene.rs:30-44's batches are independent sample ranges; only their running-mean folds are
ordered).  For N > 1 the ranks' tile radiance is gathered to rank 0 by RCCL on torch's stream
behind the last step's fold, once per frame (`--gather frame`, north_star's single frame-end
gather; the default), or after every step (`--gather step`, the reference's per-batch
read-back); the line reports the other mode beside the headline (rt_amd/shard.py FrameSteps).
`value_host_inclusive` adds one D2H copy of the final frame to the timed steps (SURVEY.md §8d:
"to final result on host"); `value` is the device-resident rate.  `bench_schema` 4: `value` is
strong scaling (since round 3) and `weak` always holds the weak-scaling figure (N = 1: the same);
the N = 1 line ends with `configs_summary`, every config's value, CPU rate and bound in one short
object (the line's tail alone shows them).  Inputs (scene, KD tree)
are resident in HBM before the timed region.  N GPUs: one process per GPU
(torch.distributed.run), image rows dealt to ranks as stripes of up to 8 rows, round-robin
(rt_amd.shard.stripe_rows).

Scaling: `value` is strong (fixed-frame) scaling — the N ranks split the W*H*spp samples of each
step, as `north_star`'s tile-parallel split of one frame asks (draw_scene.rs:17-47) and BASELINE
config 5 is (spaceship_r1 4096^2 at 1000 spp = `--scene spaceship_r1 --width 4096 --height 4096
--spp-per-step 25 --steps 40`).  For N > 1 a weak-scaling run (each rank keeps the 1-GPU step's
work: W*H/N pixels x N*spp) is reported beside it under "weak".  Either way the image is
bit-identical to the 1-GPU one (RNG and running mean are keyed on the global pixel and the
absolute sample index).

Prints ONE JSON line (rank 0).  `roofline` names the measured limiter of the trace kernel:
VALU issue (SQ_INSTS_VALU per launch over the launch's HIP-event duration, against 256 CUs x
4 SIMDs x one wave64 instruction per 2 cycles at 2.4 GHz), HBM traffic (FETCH_SIZE x 2) or, for the
mesh configs, the vector-memory issue and dependent-load latency ceilings of tools/mesh_roofline.py
(samples/s), whichever is the largest fraction; the texture units' busy fractions ride beside them.  Counter values come
from the committed rocprofv3 passes (profiles/*_counters.json) of the SAME kernel build — keyed
on a hash of the library's device code, so a kernel change without a re-profile prints null
instead of a stale figure.  SURVEY.md §8d's algorithmic bytes of the reference's traversal are
reported apart (`reference_work`): the device skips most of that work exactly, so
they are not a roofline.  `cpu_baseline` is the oracle restatement of the reference CPU renderer
on the host's cores at BASELINE.md §2's sample counts.

At N = 1 the line also carries `configs`: BASELINE.json's other single-GPU configs, each timed by
this run — a380 (10 spp in batches of 1), biplane (200 spp in batches of 10), spaceship_r1 at
4096^2 (25-spp steps: one GPU's share of config 5), and triangles (config 0, 10 spp) — each run as
render_to_target_gpu's batch loop on the device (rt_render_batches_device_async: every batch's
frame, consecutive small batches traced by one launch), with its own roofline and CPU baseline;
a380 also in a child process at HIP's default of 4 hardware queues (`hw_queues_4`).
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


def self_launch_cmd(argv, env, port):
    """The child command that runs `bench.py --gpus N` (N > 1) as N ranks when no launcher started
    this process (WORLD_SIZE unset): torch.distributed.run on one node, ranks on 127.0.0.1, the
    same arguments.  None when this process is already a rank, runs one GPU, or is bench's own
    single-process child (--config-only) or rehearsal (--as-rank)."""
    import argparse

    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config-only", default=None)
    ap.add_argument("--as-rank", default=None)
    ap.add_argument("--frame-abi", action="store_true")
    known, _ = ap.parse_known_args(argv)
    if "WORLD_SIZE" in env or known.gpus <= 1 or known.config_only or known.as_rank or known.frame_abi:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(known.gpus),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def self_launch(argv):
    """Runs self_launch_cmd's ranks as a CHILD process (subprocess: fork + exec in the child, before
    this process touches the GPU; never an exec of this process), streams the ranks' output, and
    prints rank 0's JSON line as this process's one stdout line.  Returns the exit code, or None
    when no launch is needed."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = self_launch_cmd(argv, os.environ, port)
    if cmd is None:
        return None
    env = dict(os.environ, RT_BENCH_LAUNCHER="bench.py")
    print("bench.py: --gpus > 1 without a launcher: starting " + " ".join(cmd), file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True)
    lines = []
    for ln in p.stdout:
        if ln.startswith("{"):
            lines.append(ln.strip())
        else:
            sys.stderr.write(ln)
            sys.stderr.flush()
    rc = p.wait()
    if lines:
        print(lines[-1], flush=True)
    return rc if (rc or lines) else 1


if __name__ == "__main__" and os.environ.get("WORLD_SIZE") is None:
    _rc = self_launch(sys.argv[1:])
    if _rc is not None:
        sys.exit(_rc)

# The launch pipeline's slots each want their own HIP hardware queue (launch
# pipeline): this benchmark chooses GPU_MAX_HW_QUEUES = 16 before HIP starts unless the caller
# asked for at least that, and reports what it ran with (rt_amd itself keeps explicit values).
HW_QUEUES_BEFORE = os.environ.get("GPU_MAX_HW_QUEUES")
try:
    _q = int(HW_QUEUES_BEFORE or "0")
except ValueError:
    _q = 0
# config_at_queues' child keeps the value it was given, and so do same-device test ranks (several
# processes sharing one GPU's hardware queues)
_keep = "--config-only" in sys.argv or ("--same-device" in sys.argv and HW_QUEUES_BEFORE is not None)
if _q < 16 and not _keep:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
import rt_amd  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md §L2: ~34.5 TB/s chip-wide
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 2 cycles per SIMD
# (MI355X_MICROARCH.md: SIMD-32, a wave's instruction issues over 2 cycles) at 2.4 GHz
VALU_PEAK_WINST_S = 256 * 4 * 2.4e9 / 2
# Canonical per-event byte sizes of the reference algorithm's work
BYTES = {"nodes": 8, "leaf_refs": 4, "sphere_tests": 16, "tri_tests": 36, "hits": 32, "mesh_hits": 132}
# the CPU baseline's sample count per scene (steady-state per-sample throughput)
CPU_SPP = {"walled": 20, "biplane": 10, "a380": 2, "spaceship_r1@4096": 1, "spaceship_r1": 2, "triangles": 10}
# ... over every k-th row only where a full frame takes more than ~10 s of CPU per call
CPU_ROWS_STEP = {"spaceship_r1@4096": 4}
# ... and more samples where BASELINE.md §2's count takes well under a second: each call then
# lasts a few seconds (round 4: triangles at 100 spp, 0.7-2 s per call, spread 2.1 over 3 calls)
CPU_SPP_MIN_RUN = {"triangles": 600, "a380": 8}  # a380 at 2 spp: 0.65 s per call
# BASELINE.json configs timed beside the headline at N = 1: name -> (scene, total spp, batch,
# width, height, timed repetitions of the whole config, warmup repetitions)
CONFIGS = {
    "a380": ("a380", 10, 1, None, None, 10, 1),                       # config 2: 10 spp, batch 1
    "biplane": ("biplane", 200, 10, None, None, 2, 1),                # config 3: 200 spp, batch 10
    "spaceship_r1@4096": ("spaceship_r1", 75, 25, 4096, 4096, 1, 1),  # config 5's per-GPU share: 3 steps of 25
    "triangles": ("triangles", 10, 10, None, None, 20, 2),            # config 0: 10 spp
}

from rt_amd.shard import FrameSteps, rank_tiles, step_samples, stripe_rows  # noqa: E402


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


def min_insts(scene, build_id):
    """The committed instruction floor of this kernel build on this scene (tools/min_insts.py)."""
    p = os.path.join(ROOT, "profiles", f"min_insts_{scene}.json")
    try:
        d = json.load(open(p))
    except (OSError, ValueError):
        return None
    return d, os.path.relpath(p, ROOT)


def mesh_model(config, build_id, counters, counters_src):
    """tools/mesh_roofline.py's two ceilings of the general (mesh) kernel on `config`, from the
    committed load classes of this kernel build (profiles/*_vmem_lines.jsonl) and `counters`."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import mesh_roofline

    v = mesh_roofline.vmem_entry(config, build_id)
    if not v:
        return None
    return mesh_roofline.model_from(v[0], v[1], counters, counters_src)


def roofline(scene, per_launch, kernel_ms, build_id, kernel, kernel_ms_source, model_config=None):
    """Measured fractions of the trace kernel's ceilings; bound = the largest.  For the general
    (mesh) kernel, `model_config` names its load-class measurement: the vector-memory issue and
    latency ceilings of tools/mesh_roofline.py join the candidates (mesh roofline)."""
    out = {"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": None,
           "kernel": kernel, "kernel_ms_avg": round(kernel_ms, 3), "kernel_ms_source": kernel_ms_source,
           "samples_per_launch": round(per_launch), "build_id": build_id, "counters_source": None}
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
             "insts_per_launch": d["valu_insts_per_launch"], "lane_util": d.get("valu_lane_util"),
             "wave_insts_per_sample": round(d["valu_insts_per_launch"] / per_launch, 2)}
        m = measured_valu_stream()
        if m:
            v["measured_fma_stream"] = m[0]
            v["frac_of_measured_stream"] = round(rate / 1e9 / m[0], 4)
        mi = min_insts(scene, build_id)
        if mi:
            # the instruction floor bit-exactness fixes (lane-operations per sample, every lane
            # busy) against the lane-slots the kernel actually issued per sample
            floor = mi[0]["lane_ops_per_sample"]
            issued = 64 * d["valu_insts_per_launch"] / per_launch
            v["min_lane_ops_per_sample"] = floor
            v["issued_lane_slots_per_sample"] = round(issued, 1)
            v["min_insts_frac"] = round(floor / issued, 4)
            v["min_insts_source"] = mi[1]
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
        # the texture units' busy fractions (secondary: a unit with a return outstanding counts as
        # busy, so a latency-bound kernel keeps TD busy high)
        v = {"td_busy_frac": d["td_busy_frac"], "ta_busy_frac": d.get("ta_busy_frac"),
             "note": "rocprofv3 TD_TD_BUSY_sum / TA_TA_BUSY_sum over 256 CUs x GRBM_GUI_ACTIVE / 8 XCDs, own pass; "
                     "not a bound candidate"}
        if d.get("vmem_rd_per_launch"):
            v["vmem_wave_loads_per_sample"] = round(d["vmem_rd_per_launch"] / per_launch, 2)
        out["vmem_units"] = v
    if model_config:
        m = mesh_model(model_config, build_id, d, src)
        if m:
            ach = per_launch / sec / 1e6
            for key, what in (("vmem_issue", "vector-memory issue: every load class's wave-loads at the measured "
                                             "gather cost of its shape (tools/gather_sweep.hip)"),
                              ("latency", "dependent-load chain: wave-level load steps per sample x unloaded "
                                          "latency (tools/chase_latency.hip), over the resident waves")):
                ceil = m[key]["ceiling_Msamples_s"]
                e = {"achieved": round(ach, 1), "peak": ceil, "unit": "Msamples/s", "frac": round(ach / ceil, 4),
                     "what": what}
                e.update({k: v for k, v in m[key].items() if k != "ceiling_Msamples_s"})
                out[key] = e
                fr[key] = e
            out["mesh_model"] = {"sources": m["sources"], "vmem_build_id": m["vmem_build_id"],
                                 "note": "tools/mesh_roofline.py from committed profiles; achieved = samples per launch / "
                                         "kernel_ms_avg"}
        else:
            out["mesh_model"] = {"note": f"no committed load classes of build {build_id} for {model_config}"}
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


def cgroup_cpus():
    """CPU time the cgroup lets this process use, in CPUs (cpu.max quota / period), or None."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(loaded, spp, threads=None, reps=3, rows_step=1):
    """The oracle (C++ restatement of render_to_target_cpu, recursive radiance) over the full
    frame at `spp` samples per pixel, one thread per CPU the process may use
    (the reference's rayon par_iter_mut uses all of them, draw_scene.rs:73).  The KD build and
    scene setup are timed apart (an oracle call with 0 samples), as SURVEY.md §8d asks.
    `reps` timed repetitions: the fastest is `value`, with the median / min beside it, and the
    process CPU time over each call (os.times: every thread of this process) gives the CPU the
    threads actually got — `effective_cores` = CPU-seconds / wall-seconds — and a per-core rate.
    rows_step > 1 renders every rows_step-th row only (one-row tiles over the whole frame: the
    same mix of pixels, a bounded sample of a frame too large for a few seconds of CPU)."""
    import statistics

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py  # test infrastructure: the CPU baseline leg only

    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = cgroup_cpus()
    # one thread per CPU of time the process may use: the CPUs it may run on, capped by the cgroup
    # quota (256 threads under a 16-CPU quota only contend for the same 16 CPUs' time)
    threads = threads or max(1, min(affinity, int(quota + 0.5) if quota else affinity))
    w, h = int(loaded.info.width), int(loaded.info.height)
    tiles = [(0, 0, w, h)] if rows_step <= 1 else [(0, y, w, 1) for y in range(0, h, rows_step)]
    npix = sum(t[2] * t[3] for t in tiles)

    def timed(n):
        c0, t0 = os.times(), time.perf_counter()
        oracle_py.render(loaded, tiles, 0, n, threads=threads)
        t1, c1 = time.perf_counter(), os.times()
        return t1 - t0, (c1.user - c0.user) + (c1.system - c0.system)

    timed(0)  # one-time loading
    # one untimed call at the measured spp: the first render call of a process ran at a third of
    # the later ones (round 4, triangles: 35.5 / 112.3 / 111.6 Msamples/s; thread pool and page
    # warm-up), which the median hid but the spread showed
    timed(spp)
    t_build = min(timed(0)[0], timed(0)[0])
    runs = []
    for _ in range(reps):
        wall, cpu = timed(spp)
        dt = wall - t_build
        runs.append({"Msamples_s": npix * spp / dt / 1e6, "wall_s": wall, "cpu_s": cpu,
                     "effective_cores": cpu / wall})
    vals = sorted(r["Msamples_s"] for r in runs)
    med = statistics.median(vals)
    spread = (vals[-1] - vals[0]) / med
    eff = statistics.median(r["effective_cores"] for r in runs)
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    cores = min(threads, quota) if quota else threads
    what = f"full {w}x{h} frame" if rows_step <= 1 else f"every {rows_step}th row of the {w}x{h} frame ({npix} pixels)"
    # value = the fastest call: identical calls on the box's shared host run at up to 3x different
    # rates at the same CPU-seconds, pinned or not (profiles/r5_cpu_probe_*.jsonl), so the least
    # disturbed call is the CPU's rate; it is also the baseline most favourable to the CPU
    res = {"value": round(vals[-1], 4), "unit": "Msamples/s", "cores": cores, "kind": "port",
           "reps": reps, "median": round(med, 4), "min": round(vals[0], 4), "max": round(vals[-1], 4),
           "spread": round(spread, 4),
           "effective_cores": round(eff, 2), "value_per_effective_core": round(vals[-1] / eff, 4),
           "runs": [{k: round(v, 3) for k, v in r.items()} for r in runs],
           "threads": threads, "cgroup_cpu_quota": quota, "host_cpus": os.cpu_count(), "cpu_model": model,
           "kd_build_s": round(t_build, 3),
           "sample": f"{what}, {spp} spp (BASELINE.md §2), one untimed warm-up call at that spp, then {reps} calls on "
                     f"{threads} threads, fastest call "
                     f"(KD build timed apart, CPU quota {quota or 'none'}); oracle/oracle.cpp recursive radiance; "
                     f"effective_cores = process CPU-seconds / wall-seconds of each call"}
    if spread > 0.10:
        res["spread_note"] = ("identical calls (same pixels, samples and seeds) ran at different rates with the "
                              "same CPU-seconds per call: the shared host's per-core speed varies between calls, "
                              "pinned to idle cores or not (profiles/r5_cpu_probe_*.jsonl); value is the fastest")
    return res


def kernel_label(loaded):
    """The trace kernel the scene launches (trace.hip with_queue_kernel's defaults)."""
    spheres_only = (loaded.desc.n_free_tris == 0 and loaded.desc.n_meshes == 0
                    and loaded.desc.n_spheres <= 64 and not int(loaded.info.dir_light_samp))
    dls = int(loaded.info.dir_light_samp) != 0
    restart = spheres_only or os.environ.get("RT_DEBUG_KD_RESTART", "0") not in ("0", "")
    b = lambda v: "true" if v else "false"  # noqa: E731
    return f"rtd::queue_kernel<{b(not spheres_only)}, {b(dls)}, {b(restart)}>"


def load(scene, width=None, height=None):
    from rt_amd import scheme

    sch = scheme.load_json(os.path.join(ROOT, "tests", "golden", "scenes", scene + ".json"))
    return sch, scheme.load(sch, assets_root=os.path.join(ROOT, "assets_pack"), width=width, height=height)


def sync_kernel_ms(ctx, tiles, sample, spp):
    """One synchronous call of `spp` samples: the average trace launch alone (no neighbouring
    launch overlapping it), for the roofline of pipelined (mesh) workloads."""
    ctx.render(tiles, sample, spp, want_output=False)
    ls = ctx.launch_stats()
    return ls["trace_ms"] / max(ls["n_timed_launches"], 1)


GROUP_ITEMS = 1 << 24  # rt_render_to_target's batch groups (runtime.hip GROUP_ITEMS)


def run_config(name, cpu, build_id, per_batch_calls=True):
    """One BASELINE.json config on this GPU: the whole config (its total spp in the scheme's
    batches) `reps` times after `warm` untimed runs, the way render_to_target_gpu's batch loop runs
    on the device (rt_render_batches_device_async: batch k's frame into its own buffer, consecutive
    batches traced together in groups of up to GROUP_ITEMS samples, as rt_render_to_target groups
    them).  Beside it: the same config as one async call per batch (rt_render_device_async, the
    round-3 method, which needs a hardware queue per batch in flight), and the host-inclusive rate
    (the last frame copied to host memory inside the timed region).  Then the roofline of its
    trace launches and the CPU baseline at BASELINE.md §2's spp."""
    import torch

    from rt_amd import render

    scene, total, batch, width, height, reps, warm = CONFIGS[name]
    _, loaded = load(scene, width, height)
    w, h = int(loaded.info.width), int(loaded.info.height)
    tiles = [(0, 0, w, h)]
    nb = total // batch
    group_items = GROUP_ITEMS  # as rt_render_to_target reads it (RT_DEBUG_LAUNCH group_items overrides)
    for kv in os.environ.get("RT_DEBUG_LAUNCH", "").split(","):
        if kv.startswith("group_items="):
            group_items = int(kv.split("=", 1)[1])
    group = max(1, min(nb, group_items // (w * h * batch)))
    res = {"workload": f"{scene}.yml {w}x{h}, {total} spp in batches of {batch}, kd_tree_depth "
                       f"{int(loaded.info.kd_tree_depth)}; {nb} batches per run, each batch's frame in its own "
                       f"device buffer, traced {group} batches per launch"}
    with render.Context(loaded) as ctx:
        outs = [torch.zeros((w * h, 4), dtype=torch.float32, device="cuda:0") for _ in range(nb)]
        stream = torch.cuda.current_stream().cuda_stream
        sample = 0

        def whole_batches():
            nonlocal sample
            for g0 in range(0, nb, group):
                ptrs = [o.data_ptr() for o in outs[g0:g0 + group]]
                ctx.render_batches_device_async(ptrs, tiles, sample, batch, stream=stream)
                sample += batch * len(ptrs)

        def whole_calls():
            nonlocal sample
            for k in range(nb):
                ctx.render_device_async(outs[k].data_ptr(), tiles, sample, batch, stream=stream)
                sample += batch

        def timed(fn):
            for _ in range(warm):
                fn()
            ctx.synchronize()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            ctx.synchronize()
            torch.cuda.synchronize()
            return time.perf_counter() - t0, ctx.launch_stats()

        elapsed, ls = timed(whole_batches)
        # the final result on the host: the last frame's D2H copy, timed after the run
        t0 = time.perf_counter()
        last = outs[nb - 1].cpu()
        elapsed_host = elapsed + time.perf_counter() - t0
        del last
        # one call per batch only differs when batches are grouped
        per_calls = timed(whole_calls)[0] if per_batch_calls and group > 1 else None
        per_launch = w * h * batch * group
        kms = sync_kernel_ms(ctx, tiles, sample, batch * group)
        ok = bool((outs[nb - 1][:, 3] == 1.0).all().item())
    rate = lambda t: round(w * h * total * reps / t / 1e6, 3)  # noqa: E731
    res.update(value=rate(elapsed), unit="Msamples/s", spp=total, batch=batch, batches_per_launch=group, reps=reps,
               elapsed_s=round(elapsed, 4), frame_complete=ok, value_host_inclusive=rate(elapsed_host),
               launch={"trace_launches": ls["n_trace_launches"], "samples_per_launch": per_launch,
                       "trace_ms_per_launch_overlapped": round(ls["trace_ms"] / max(ls["n_timed_launches"], 1), 3),
                       "trace_ms_per_launch_sync": round(kms, 3)})
    if per_calls is not None:
        res["value_per_batch_calls"] = rate(per_calls)
    res["roofline"] = roofline(scene if name != "spaceship_r1@4096" else "spaceship_r1", per_launch, kms, build_id,
                               kernel_label(loaded), "one synchronous launch (no overlap)", model_config=name)
    if cpu:
        res["cpu_baseline"] = cpu_baseline(loaded, CPU_SPP_MIN_RUN.get(name, CPU_SPP[name]),
                                           rows_step=CPU_ROWS_STEP.get(name, 1))
        res["speedup_vs_cpu"] = round(res["value"] / res["cpu_baseline"]["value"], 1)
    return res


def config_at_queues(name, queues):
    """run_config in a child process that starts HIP with GPU_MAX_HW_QUEUES = `queues` (HIP reads
    it once, at start): what a caller who leaves HIP's default of 4 gets.  The child is started
    with subprocess (fork + exec before it touches the GPU), never by replacing this process."""
    import subprocess

    env = dict(os.environ, GPU_MAX_HW_QUEUES=str(queues))
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--config-only", name], env=env,
                       capture_output=True, text=True, timeout=600)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode or not line:
        return {"error": (r.stderr or r.stdout)[-500:]}
    d = json.loads(line[-1])
    return {k: d[k] for k in ("value", "value_per_batch_calls", "hw_queues") if k in d}


def device_identity(rank, local):
    """Which GPU this rank runs on: its device ordinal, PCI location (domain:bus:device, as
    hipDeviceGetPCIBusId prints it) and UUID, so an N-rank line shows the ranks on N devices."""
    import torch

    p = torch.cuda.get_device_properties(local)
    return {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "device": local,
            "pci_bus_id": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0",
            "uuid": str(getattr(p, "uuid", "")), "name": p.name, "arch": getattr(p, "gcnArchName", ""),
            "visible_devices": os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")}


def gather_identities(ident, dist, world):
    """Every rank's device_identity, on every rank (all_gather_object over the process group)."""
    if dist is None:
        return [ident]
    out = [None] * world
    dist.all_gather_object(out, ident)
    return out


def rank_summary(idents, dist):
    """The N-rank line's proof of what ran: each rank's device and PCI location, how many distinct
    devices they were, and the process group's backend and size."""
    r = {"ranks": idents, "distinct_devices": len({i["pci_bus_id"] + i["uuid"] for i in idents})}
    if dist is not None:
        r["dist"] = {"backend": dist.get_backend(), "world_size": dist.get_world_size()}
    return r


def frame_abi_run(loaded, devices, spp, steps, warmup, digest=False):
    """The C-ABI multi-device frame (rt_frame_*, frame.hip) in THIS process: one context per entry
    of `devices` (each renders its stripes, the deal of rt_stripe_tiles), `warmup` untimed steps,
    then exactly `steps` steps of `spp` samples over the whole frame (strong scaling: the contexts
    split each step's W*H*spp samples) and ONE gather at the frame's end (peer copies to devices[0],
    then one placement per context), synchronized on every device before and after.  This is the
    path the reference's render thread (renderer.rs:43-60) would call; bench.py's torch ranks
    measure the same split with one process per GPU."""
    import hashlib

    import torch

    from rt_amd import render

    w, h = int(loaded.info.width), int(loaded.info.height)
    with render.Frame(loaded, devices) as f:
        s0 = 0
        for _ in range(warmup):
            f.render(s0, spp)
            s0 += spp
        f.gather(want_host=False)
        f.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            f.render(s0, spp)
            s0 += spp
        f.gather(want_host=False)  # the frame-end gather (returns once the frame is placed)
        f.synchronize()
        dt = time.perf_counter() - t0
        st = f.stats()
        out = {"value": round(w * h * spp * steps / dt / 1e6, 3), "unit": "Msamples/s",
               "ms_per_step": round(dt / steps * 1e3, 3), "devices": list(devices),
               "pci_bus_ids": [device_identity(0, d)["pci_bus_id"] for d in sorted(set(devices))],
               "stripe_rows": st["stripe_rows"], "gathers_timed": 1,
               "peer_copy_ms_max": round(st["peer_copy_ms_max"], 3), "place_ms": round(st["place_ms"], 3),
               "render_ms_max": round(st["render_ms_max"], 3), "n_peer_copies": st["n_peer_copies"],
               "n_parts": st["n_parts"],
               "note": "rt_frame_* in one process (C ABI, frame.hip): one context per device, one gather per frame "
                       "(hipMemcpyPeerAsync to the first device + one strided placement per context)"}
        if digest:
            frame = f.gather(want_host=True)  # after the timed region
            out["frame_sha256"] = hashlib.sha256(frame.tobytes()).hexdigest()
            out["frame_complete"] = bool((frame[..., 3] == 1.0).all())
    torch.cuda.synchronize()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scene", default="walled")
    ap.add_argument("--spp-per-step", type=int, default=None,
                    help="samples per pixel per step (default: the scheme's gpu_render_batch)")
    ap.add_argument("--width", type=int, default=None, help="override the scheme's width")
    ap.add_argument("--height", type=int, default=None, help="override the scheme's height")
    ap.add_argument("--weak", action="store_true", help="weak scaling as the headline (each rank N*spp)")
    ap.add_argument("--strong", action="store_true", help="(the default) fixed frame: N ranks split W*H*spp")
    ap.add_argument("--sync", action="store_true", help="synchronous steps (rt_render_device), for A/B")
    ap.add_argument("--cpu-threads", type=int, default=None)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-configs", action="store_true", help="skip the other BASELINE configs (N = 1)")
    ap.add_argument("--stripe", type=int, default=None,
                    help="rows per stripe (default: rt_amd.shard.stripe_rows, equal stripe counts per rank)")
    ap.add_argument("--as-rank", default=None,
                    help="r/N: time rank r's share of an N-GPU run on this one GPU (no gather); "
                         "a scaling rehearsal, not the contract's multi-process run")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="gloo: gather host copies (multi-rank test with every rank on one GPU)")
    ap.add_argument("--same-device", action="store_true", help="every rank on device 0 (tests; gloo only)")
    ap.add_argument("--dump-frame", default=None, help="rank 0 saves the last assembled frame (.npy)")
    ap.add_argument("--frame-digest", action="store_true",
                    help="rank 0 adds the sha256 of every run's assembled frame (headline, other gather mode, "
                         "weak / strong) to the line: bit-equality checks of large frames without dumping them")
    ap.add_argument("--gather", default="frame", choices=("frame", "step"),
                    help="N > 1: gather the ranks' tiles once at frame end (north_star; default) or after every "
                         "step (the reference's per-batch read-back); the other mode is reported beside it")
    ap.add_argument("--frame-abi", action="store_true",
                    help="time the C-ABI multi-device frame (rt_frame_*: one process, one context per device, "
                         "one gather per frame) as the headline instead of torch ranks; --gpus N contexts")
    ap.add_argument("--frame-devices", default=None,
                    help="comma-separated device ordinals of the --frame-abi contexts (default 0..N-1; tests: 0,0)")
    ap.add_argument("--no-frame-abi", action="store_true",
                    help="N > 1 torch ranks: skip rank 0's C-ABI frame leg over the ranks' devices")
    ap.add_argument("--config-only", default=None, choices=sorted(CONFIGS),
                    help="print one BASELINE config's JSON (no CPU leg) and exit: bench's child for the "
                         "4-queue a380 figure")
    args = ap.parse_args()
    if args.config_only:
        r = run_config(args.config_only, False, None)
        r["hw_queues"] = os.environ.get("GPU_MAX_HW_QUEUES")
        print(json.dumps(r), flush=True)
        return
    if args.same_device and args.dist_backend != "gloo":
        raise SystemExit("--same-device needs --dist-backend gloo (RCCL refuses two ranks on one GPU)")
    if args.frame_abi:
        return main_frame_abi(args)

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    # a host-side group for waits that must not hold a GPU: an RCCL barrier keeps a collective
    # kernel spinning on every waiting rank's GPU (rank 0's C-ABI leg below uses those GPUs)
    cpu_pg = dist.new_group(backend="gloo") if dist is not None and args.dist_backend == "nccl" else None

    from rt_amd import abi, render

    # every rank's device, gathered to rank 0: the line shows which GPUs the N ranks ran on
    idents = gather_identities(device_identity(rank, local), dist, world)
    sch, loaded = load(args.scene, args.width, args.height)
    w, h = int(loaded.info.width), int(loaded.info.height)
    spp = args.spp_per_step or int(sch["render_info"].get("gpu_render_batch") or 1)
    shard_rank, shard_world = rank, world
    if args.as_rank:
        if world != 1:
            raise SystemExit("--as-rank is a single-process rehearsal")
        shard_rank, shard_world = (int(v) for v in args.as_rank.split("/"))
    stripe = args.stripe or stripe_rows(h, shard_world)
    tiles = rank_tiles(w, h, shard_rank, shard_world, stripe)
    strong = not args.weak

    ctx = render.Context(loaded, device=local)

    def timed_run(strong_mode, gather):
        spp_rank, job_samples = step_samples(w, h, spp, shard_world, strong_mode)
        fs = FrameSteps(ctx, tiles, w, h, rank, world, stripe, spp_rank, local, dist=dist,
                        backend=args.dist_backend, sync=args.sync, gather=gather)
        r = fs.run(args.steps, args.warmup)
        if args.as_rank:
            job_samples = fs.npix * spp_rank  # one rank's share only
        r.update(spp_rank=spp_rank, npix=fs.npix, value=job_samples * args.steps / r["elapsed_s"] / 1e6,
                 value_host_inclusive=job_samples * args.steps / (r["elapsed_s"] + r["host_copy_s"]) / 1e6)
        return fs, r

    def digest(fs):
        """rank 0: sha256 of the assembled frame's bytes (None elsewhere / when not asked)."""
        if not args.frame_digest or args.as_rank or rank != 0:
            return None
        import hashlib

        import numpy as np

        return hashlib.sha256(np.ascontiguousarray(fs.frame(), dtype=np.float32).tobytes()).hexdigest()

    fs, r = timed_run(strong, args.gather)
    elapsed, ls, spp_rank, npix = r["elapsed_s"], r["launch"], r["spp_rank"], r["npix"]
    # after the timed region: rank 0 reassembles the last gathered frame and checks that every
    # pixel was rendered by some rank (alpha is 1 exactly where written)
    frame_complete = None
    frame_sha = digest(fs)
    if not args.as_rank and rank == 0:
        frame = fs.frame()
        frame_complete = bool((frame[..., 3] == 1.0).all())
        if args.dump_frame:
            import numpy as np

            np.save(args.dump_frame, frame)
        del frame
    del fs

    n_launch = ls["n_trace_launches"]
    per_launch = npix * spp_rank * args.steps / max(n_launch, 1)
    kernel_ms = ls["trace_ms"] / max(ls.get("n_timed_launches", n_launch), 1)
    res = {"metric": f"Msamples/s (pixels x spp / s) on {args.scene}.yml",
           "value": round(r["value"], 3), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
           "bench_schema": 4,
           "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
           "higher_is_better": True, "scaling": "strong" if strong else "weak", "vs_baseline": None,
           "dtype": "f32",
           "data": "synthetic-free: the reference's own scene file (tests/golden/scenes), seeded RNG",
           "config": {"workload": f"{args.scene}.yml {w}x{h}, {spp} spp per step"
                                  f"{'' if strong else ' x n_gpus'} (one queue launch per rank and step), "
                                  f"kd_tree_depth {int(loaded.info.kd_tree_depth)}",
                      "spp_per_step": spp, "pixels": w * h, "stripes": f"{stripe}-row round-robin",
                      "parallelism": f"tiles{world}", "dispatch": "sync" if args.sync else "async",
                      "dist_backend": args.dist_backend if world > 1 else None}}
    res["frame_complete"] = frame_complete
    res.update(rank_summary(idents, dist))
    if frame_sha:
        res["frame_sha256"] = frame_sha
    res["launcher"] = (os.environ.get("RT_BENCH_LAUNCHER") or "torch.distributed.run") if world > 1 else None
    # the final frame on the host (SURVEY.md §8d "to final result on host"): one D2H copy of the
    # (gathered) frame after the timed steps, added to their time; `value` stays device-resident
    res["value_host_inclusive"] = round(r["value_host_inclusive"], 3)
    res["host_copy_ms"] = round(r["host_copy_s"] * 1e3, 3)
    res["launch"] = {"trace_launches_per_step": n_launch / args.steps, "samples_per_launch": round(per_launch),
                     "trace_ms_per_launch": round(kernel_ms, 3),
                     "device_window_ms": round(ls["render_ms"], 3)}
    res["hw_queues"] = {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"), "caller_value": HW_QUEUES_BEFORE,
                        "hip_started_before_rt_amd": rt_amd.hw_queues()["hip_started_before_import"]}
    if "gather_ms_per_step" in r:
        res["gather"] = {"mode": r["gather_mode"], "gathers": r["gathers"],
                         "ms_per_gather": round(r["gather_ms_per_gather"], 3)}
        res["gather_ms_per_step"] = round(r["gather_ms_per_step"], 3)
    if args.as_rank:
        res["config"]["rehearsal"] = f"rank {shard_rank} of {shard_world}, single GPU, no gather"
        res["scaling"] = None
    if world > 1:
        # the other gather mode (frame end <-> every step), same scaling as the headline
        other = "step" if args.gather == "frame" else "frame"
        fg, rg = timed_run(strong, other)
        res[f"gather_{other}"] = {
            "value": round(rg["value"], 3), "ms_per_step": round(rg["elapsed_s"] / args.steps * 1e3, 3),
            "gathers": rg["gathers"], "ms_per_gather": round(rg.get("gather_ms_per_gather", 0.0), 3),
            "gather_ms_per_step": round(rg.get("gather_ms_per_step", 0.0), 3)}
        if args.frame_digest and rank == 0:
            res[f"gather_{other}"]["frame_sha256"] = digest(fg)
        del fg
        # weak scaling beside the strong headline (each rank keeps the 1-GPU step's work)
        fw, rw = timed_run(not strong, args.gather)
        res["weak" if strong else "strong"] = {
            "value": round(rw["value"], 3), "ms_per_step": round(rw["elapsed_s"] / args.steps * 1e3, 3),
            "spp_per_rank_step": rw["spp_rank"], "gather_ms_per_step": round(rw.get("gather_ms_per_step", 0.0), 3)}
        if args.frame_digest and rank == 0:
            res["weak" if strong else "strong"]["frame_sha256"] = digest(fw)
        del fw
    elif not args.as_rank:
        res["weak"] = {"value": res["value"], "note": "N = 1: weak and strong scaling are the same run"}
    if world > 1 and not args.no_frame_abi:
        # the same strong split through the C ABI (rt_frame_*): rank 0 alone, one context on each
        # rank's device, while the other ranks wait at a barrier
        torch.cuda.synchronize()
        dist.barrier(group=cpu_pg)
        if rank == 0:
            try:
                res["frame_abi"] = frame_abi_run(loaded, [i["device"] for i in idents], spp, args.steps,
                                                 args.warmup, digest=args.frame_digest)
            except Exception as e:  # reported, never fatal to the torch-rank headline
                res["frame_abi"] = {"error": repr(e)[:300]}
        dist.barrier(group=cpu_pg)

    build_id = abi.kernel_build_id()
    if rank == 0 and not args.no_roofline:
        res["roofline"] = roofline(args.scene, per_launch, kernel_ms, build_id, kernel_label(loaded),
                                   "HIP events around each trace launch of the timed steps")
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
        # north_star's ">= 40% of HBM-read roofline in the traversal loop": not a gate this kernel can be
        # scored on, and the line says so
        hbm = res["roofline"].get("hbm") or {}
        res["north_star_hbm_gate"] = {
            "reference_algorithm_GB_s": res["reference_work"]["GB_s"],
            "reference_algorithm_frac_of_peak": round(res["reference_work"]["GB_s"] / HBM_PEAK_GBS, 2),
            "measured_hbm_frac": hbm.get("frac"),
            "scored": False,
            "why": "the reference's traversal bytes at this rate would exceed the 8 TB/s peak (frac > 1): the "
                   "device does not do that work (it skips it exactly), and what it does read hits L2/MALL, so HBM "
                   "is a few percent busy; the kernel's measured limiter is `roofline.bound`"}
    ctx.close()
    single = rank == 0 and world == 1 and not args.as_rank
    if single and not args.no_cpu:
        cs = CPU_SPP.get(args.scene if not (args.width or args.height) else args.scene + f"@{w}", 2)
        res["cpu_baseline"] = cpu_baseline(loaded, cs, args.cpu_threads)
        res["speedup_vs_cpu"] = round(res["value"] / res["cpu_baseline"]["value"], 1)
    if single and not args.no_configs and args.scene == "walled":
        res["configs"] = {}
        for name in CONFIGS:
            res["configs"][name] = run_config(name, not args.no_cpu, build_id)
        # config 2 as a caller that leaves HIP's default of 4 hardware queues gets it
        res["configs"]["a380"]["hw_queues_4"] = config_at_queues("a380", 4)
        # the configs' headline numbers once more, compactly, as the line's last key: a reader of
        # only the line's tail still sees every config's value
        res["configs_summary"] = {n: {"value": c.get("value"), "value_host_inclusive": c.get("value_host_inclusive"),
                                      "cpu": (c.get("cpu_baseline") or {}).get("value"),
                                      "bound": (c.get("roofline") or {}).get("bound"),
                                      "frac": (c.get("roofline") or {}).get("frac")}
                                  for n, c in res["configs"].items()}
        res["configs_summary"]["a380"]["value_at_4_hw_queues"] = res["configs"]["a380"]["hw_queues_4"].get("value")
        res["configs_summary"]["walled"] = {"value": res["value"], "value_host_inclusive": res.get("value_host_inclusive"),
                                            "cpu": (res.get("cpu_baseline") or {}).get("value"),
                                            "bound": (res.get("roofline") or {}).get("bound"),
                                            "frac": (res.get("roofline") or {}).get("frac")}
    if dist:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(res), flush=True)


def main_frame_abi(args):
    """`--frame-abi`: the headline is the C-ABI multi-device frame in one process (no torch ranks,
    no launcher): --gpus N contexts on --frame-devices (default 0..N-1), strong scaling."""
    import torch

    from rt_amd import abi

    devices = ([int(d) for d in args.frame_devices.split(",")] if args.frame_devices else list(range(args.gpus)))
    if len(devices) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but {len(devices)} --frame-devices")
    torch.cuda.set_device(devices[0])
    sch, loaded = load(args.scene, args.width, args.height)
    w, h = int(loaded.info.width), int(loaded.info.height)
    spp = args.spp_per_step or int(sch["render_info"].get("gpu_render_batch") or 1)
    r = frame_abi_run(loaded, devices, spp, args.steps, args.warmup, digest=args.frame_digest)
    res = {"metric": f"Msamples/s (pixels x spp / s) on {args.scene}.yml", "value": r["value"], "unit": "Msamples/s",
           "n_gpus": args.gpus, "steps": args.steps, "warmup": args.warmup, "ms_per_step": r["ms_per_step"],
           "bench_schema": 4, "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
           "data": "synthetic-free: the reference's own scene file (tests/golden/scenes), seeded RNG",
           "config": {"workload": f"{args.scene}.yml {w}x{h}, {spp} spp per step, split over {args.gpus} "
                                  f"contexts of one process (rt_frame_*)", "spp_per_step": spp, "pixels": w * h,
                      "parallelism": f"frame_abi{args.gpus}", "dispatch": "async"},
           "frame_abi": r, "ranks": [device_identity(0, d) for d in devices],
           "distinct_devices": len(set(devices)), "build_id": abi.kernel_build_id()}
    if "frame_sha256" in r:
        res["frame_sha256"] = r["frame_sha256"]
        res["frame_complete"] = r["frame_complete"]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
