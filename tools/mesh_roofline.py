#!/usr/bin/env python3
"""Throughput ceilings of the general (mesh) queue kernel, from committed measurements only
("Mesh roofline").  Two ceilings in samples/s, each with every input and its source:

1. Vector-memory issue.  Each class c of the kernel's vector loads (tools/vmem_classes.py: wave-loads
   wl_c and distinct 128-B lines per sample, diag build of the same source) costs the chip the time
   the gather microbenchmark measured for a wave-load of that shape (tools/gather_rates.hip,
   profiles/r2_gather_rates.json: record size x lines per wave-load, interpolated in time per
   wave-load between the measured "same" (1 line), "runs16" and "random" (64 lines) patterns),
   blended between the L1-resident and the L2-resident table by the kernel's L1 line hit fraction
   h1 = 1 - (L2 requests per sample, rocprofv3 TCC counters of the product build) / (distinct lines
   per sample):  T_v = sum_c wl_c (h1 / R_L1(c) + (1 - h1) / R_L2(c)),  ceiling_v = 1 / T_v.
2. Latency.  Each wave runs its cooperative rounds as a chain of dependent loads: per sample S
   wave-level steps (a descent load per node level; two per
   cooperative pass, ref then triangle; two per winner re-test and leading-sphere test; one per
   path start, shading record and texel fetch), each at least the unloaded latency of one
   dependent load (tools/chase_latency.hip, profiles/r5_chase_latency.jsonl: random lanes, 8 KiB /
   3 MiB / 32 MiB working sets for L1 / L2 / MALL), weighted by h1 and the L2 hit rate.  With W
   resident waves (256 CUs x 4 SIMDs x 8):  ceiling_l = W / (S x L).

The bench line reports achieved / ceiling for both and names the tighter (the larger fraction) as
`roofline.bound`, with the texture units' busy fractions beside them.
Usage: python tools/mesh_roofline.py > profiles/<tag>_mesh_roofline.json"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")

# record kind of each load class: bytes per lane of one wave-load (trace.hip)
KIND = {"descent": "dwordx4", "pop": "dwordx2", "pass_ref": "dword", "pass_tri": "dwordx4", "lead_sph": "dwordx4",
        "retest": "dwordx4", "pixq": "dwordx4", "mesh_rec": "dwordx4", "tex": "dword"}
# distinct 128-B lines of one "runs16" wave-load (4 runs of 16 consecutive records)
RUNS16_LINES = {"dword": 4, "dwordx2": 4, "dwordx3": 8, "dwordx4": 8}
RESIDENT_WAVES = 256 * 4 * 8  # general queue kernel: 8 waves per SIMD (RT_MIN_WAVES_GEN)


def gather_table():
    """{(kind, level): [(lines, ns per wave-load chip-wide)]} from r2_gather_rates.json; level 'L1' is
    the smallest table, 'L2' the largest."""
    rows = [json.loads(l) for l in open(os.path.join(PROF, "r2_gather_rates.json")) if l.strip()]
    by = {}
    for r in rows:
        if r["layout"] not in RUNS16_LINES:
            continue
        by.setdefault(r["layout"], {}).setdefault(r["table_KiB"], {})[r["pattern"]] = 1.0 / r["G_wave_loads_per_s"]
    out = {}
    for kind, tabs in by.items():
        for level, kib in (("L1", min(tabs)), ("L2", max(tabs))):
            t = tabs[kib]
            out[(kind, level)] = [(1, t["same"]), (RUNS16_LINES[kind], t["runs16"]), (64, t["random"])]
    return out


def sweep_table():
    """{(kind, level, active_lanes): [(lines per wave-load, ns per wave-load chip-wide)]} from the
    committed gather sweep (tools/gather_sweep.hip), or None when there is none."""
    files = sorted(glob.glob(os.path.join(PROF, "*_gather_sweep.jsonl")))
    if not files:
        return None, None
    out = {}
    for line in open(files[-1]):
        if not line.strip():
            continue
        r = json.loads(line)
        level = "L1" if r["table_KiB"] <= 32 else "L2"
        out.setdefault((r["kind"], level, r["active_lanes"]), []).append(
            (r["lines_per_wave_load"], 1.0 / r["G_wave_loads_per_s"]))
    for k in out:
        out[k].sort()
    return out, os.path.relpath(files[-1], ROOT)


def sweep_cost(table, kind, level, lanes, lines):
    """ns per wave-load of `kind` with `lanes` active lanes touching `lines` lines: interpolated in
    lines on each measured active-lane curve, then linearly between the two nearest lane counts."""
    curves = sorted(a for (k, lv, a) in table if k == kind and lv == level)
    lanes = min(max(lanes, curves[0]), curves[-1])
    lo = max(a for a in curves if a <= lanes)
    hi = min(a for a in curves if a >= lanes)
    tlo = interp(table[(kind, level, lo)], lines)
    if hi == lo:
        return tlo
    thi = interp(table[(kind, level, hi)], lines)
    return tlo + (thi - tlo) * (lanes - lo) / (hi - lo)


def interp(points, x):
    x = min(max(x, points[0][0]), points[-1][0])
    for (x0, y0), (x1, y1) in zip(points, points[1:]):
        if x <= x1:
            return y0 + (y1 - y0) * (x - x0) / (x1 - x0)
    return points[-1][1]


def chase_latency():
    rows = [json.loads(l) for l in open(os.path.join(PROF, "r5_chase_latency.jsonl")) if l.strip()]
    rnd = {r["working_set_bytes"]: r["ns_per_step"] for r in rows if r["lanes"] == "64 random"}
    return {"L1": rnd[8192], "L2": rnd[3145728], "MALL": rnd[33554432]}


def vmem_entry(config, build_id=None):
    """The latest committed load-class measurement of `config` (tools/vmem_classes.py; spaceship_r1@4096
    for the 4096 x 4096 frame), of the product build `build_id` when given."""
    best = None
    for p in sorted(glob.glob(os.path.join(PROF, "*_vmem_lines.jsonl"))):
        for line in open(p):
            if not line.strip():
                continue
            d = json.loads(line)
            if d.get("config", d.get("scene")) != config or "lines_by_class" not in d:
                continue
            if build_id is not None and d.get("build_id") != build_id:
                continue
            if d.get("treelet", "0") not in ("0", ""):
                continue  # round 6's treelet experiment (profiles/r6_ab/treelet_*), not the product kernel
            best = (d, os.path.relpath(p, ROOT))
    return best


def counters_for(scene, build_id=None):
    best = None
    for p in sorted(glob.glob(os.path.join(PROF, "*_counters.json"))):
        d = json.load(open(p))
        if d.get("scene") == scene and d.get("l2_bytes_per_launch") and (build_id is None or d.get("build_id") == build_id):
            best = (d, os.path.relpath(p, ROOT))
    return best


def model_from(vl, vsrc, cnt, csrc):
    """The two ceilings from one load-class measurement (vl) and the product build's counters (cnt)."""
    per, cls = vl["per_sample"], vl["lines_by_class"]
    gt = gather_table()
    sw, sw_src = sweep_table()
    lines_total = sum(x["lines_128"] for x in cls.values())
    l2_req = cnt["l2_bytes_per_launch"] / 128.0 / cnt["samples_per_launch"]
    h1 = min(1.0, max(0.0, 1.0 - l2_req / lines_total))
    classes, t_v = {}, 0.0
    for name, x in cls.items():
        wl = per.get(name, 0.0)
        if not wl:
            continue
        kind = KIND[name]
        n = x["lines_128"] / wl
        lanes = x["lanes"] / wl  # active lanes per wave-load (one VL per wave-load)
        if sw:
            sk = "tri48" if name in ("pass_tri", "retest", "lead_sph") else kind
            t1, t2 = sweep_cost(sw, sk, "L1", lanes, n), sweep_cost(sw, sk, "L2", lanes, n)
        else:
            t1, t2 = interp(gt[(kind, "L1")], n), interp(gt[(kind, "L2")], n)
        t = wl * (h1 * t1 + (1.0 - h1) * t2)
        t_v += t
        classes[name] = {"wave_loads": wl, "kind": kind, "lines_per_wave_load": round(n, 2),
                         "active_lanes": round(lanes, 1),
                         "ns_L1": round(t1, 5), "ns_L2": round(t2, 5), "ns_per_sample": round(t, 4)}
    steps = {"descent": per["descent"],
             "passes": 2.0 * per["passes"], "retest": 2.0 * per["retest"] / 4.0, "lead_sph": per["lead_sph"],
             "pixq": per["pixq"], "mesh_rec": per["mesh_rec"], "tex": per["tex"]}
    s = sum(steps.values())
    lat = chase_latency()
    l2h = cnt.get("l2_hit_rate") or 0.0
    lat_ns = h1 * lat["L1"] + (1 - h1) * (l2h * lat["L2"] + (1 - l2h) * lat["MALL"])
    return {"config": vl.get("config", vl.get("scene")),
            "vmem_issue": {"ns_per_sample": round(t_v, 4), "ceiling_Msamples_s": round(1e3 / t_v, 1),
                           "l1_line_hit_frac": round(h1, 4), "l2_requests_per_sample": round(l2_req, 2),
                           "distinct_lines_per_sample": round(lines_total, 2), "classes": classes},
            "latency": {"steps_per_sample": round(s, 3), "steps": {k: round(x, 3) for k, x in steps.items()},
                        "ns_per_step": round(lat_ns, 2), "resident_waves": RESIDENT_WAVES,
                        "ceiling_Msamples_s": round(RESIDENT_WAVES / (s * lat_ns) * 1e3, 1),
                        "latency_ns": lat, "l2_hit_rate": l2h},
            "sources": {"vmem_classes": vsrc, "counters": csrc,
                        "gather_rates": sw_src if sw else "profiles/r2_gather_rates.json",
                        "chase_latency": "profiles/r5_chase_latency.jsonl"},
            "counters_build_id": cnt.get("build_id"), "vmem_build_id": vl.get("build_id"),
            "vmem_spp_per_launch": vl.get("spp_per_launch")}


def model(config, build_id=None):
    scene = config.split("@")[0]
    v = vmem_entry(config, build_id)
    c = counters_for(scene, build_id)
    if not v or not c:
        return None
    return model_from(v[0], v[1], c[0], c[1])


def main(argv):
    for config in argv or ("a380", "biplane", "spaceship_r1@4096", "triangles"):
        m = model(config)
        print(json.dumps(m if m else {"config": config, "error": "no load classes or counters"}), flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
