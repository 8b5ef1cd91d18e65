"""The instruction floor of the sphere-only trace kernel (walled.yml): the lane-operations per
sample that bit-exactness fixes, against which bench.py sets the VALU instructions the kernel
actually issues (roofline.valu.min_insts_frac).

A lane-operation is one f32 / integer operation of the reference's own arithmetic on one lane:
each IEEE add, mul, compare, select, division and square root counts 1, the glibc sinf/cosf/powf
restatements their polynomial and reduction steps, 64-bit integer work its 32-bit parts.  Loads,
address arithmetic, loop control, the exactness guards and the queue bookkeeping are not in the
floor.  The per-event counts come from the oracle's instrumented render of the reference algorithm
on the bench's scene (every 16th pixel in x and y, 16 spp, SURVEY.md §8d's grid): segments,
sphere hits, spheres whose discriminant is positive, continued rays by material branch,
Russian-roulette draws and all draws.  The closest-hit floor is the device algorithm's
(closest_small: every sphere's discriminant, the roots of every sphere the ray's line meets,
the in_return_leaf decision), which returns the reference's sphere and length exactly
(DESIGN.md §5); the reference's own traversal costs far more (507 node steps).

Usage: python tools/min_insts.py [scene] -> profiles/min_insts_<scene>.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("gpu-ray_trace-rust_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))

# lane-operations per event (trace.hip / rt_rng.h / rt_libm.h; see the comments for each)
OPS = {
    # per sample: stream start mix64(key ^ sample) = 64-bit xor (2), three shift-xor rounds (4
    # each), two 64x64 multiplies by constants (6 each), the zero-state guard (2); pixel x, y
    # from the table word (2);
    # camera_base_dir: 2 x (cvt, sub, mul) + 6 mul + 6 add; jitter: 2 sub, 12 mul, 6 add; the
    # fold: 3 x (mul, add, div), n + 1, cvt n
    "sample": 26 + 2 + 2 + 18 + 20 + 11,
    # per draw (rt_rng_next_f32): xoroshiro64* (round 4): the output multiply, s1 ^ s0, two
    # rotates, s1 << 9, two xors; >> 8, cvt, * 2^-24
    "draw": 7 + 3,
    # per segment: normalize the direction (dot 5, sqrt, 3 div)
    "segment": 9,
    # per sphere and segment: sphere_disc, o - c (3), two dots (10), - r^2, dir^2 - consts (2),
    # the thing2 > 0 test
    "sphere_disc": 17,
    # per sphere whose discriminant is positive (the ray's line meets it): its roots and the
    # running minimum (sqrt, -dir, two adds, l1 > 0, select, l >= HIT_MIN, l < best, two
    # selects); the closest hit needs every such sphere's length
    "sphere_roots": 10,
    # per segment that hits: in_return_leaf (round 6: it stands in for the root slab test) — the
    # two thresholds 2, per axis a reciprocal, two face differences and two products 15, near and
    # far per axis and their max / min over the axes 10, two compares 2
    "hit_segment": 2 + 15 + 10 + 2,
    # per sphere hit: hit_info (perfect 6, normalize(perfect - c) 12, pos 6), emission 6, T *= rgb
    # * p 6, d.n 5, the mirror direction 9
    "hit": 24 + 6 + 6 + 5 + 9,
    # per diffuse continue (interaction.rs:11-27): xd 15, yd 18, sqrt(u), 2 pi v, sincos (cvt,
    # reduction, two short f64 polynomials, cvt back: 17), x, y (2), the new direction 17
    "diff": 15 + 18 + 1 + 1 + 17 + 2 + 17,
    # per refracting continue (interaction.rs:29-59): into / c1 / normal / n_over 7, c22 5,
    # sqrt, compare, trns 11, c 3, powf(c, 5) ~20, re 3, the draw's compare and p 2
    "dielectric": 7 + 5 + 1 + 1 + 11 + 3 + 20 + 3 + 2,
    # per DiffSpec seed (uniform_diff_spec.rs:33-36): the compare
    "diffspec_seed": 1,
    # per Russian-roulette draw (radiance.rs:74-86): depth compare, draw compare
    "rr": 2,
}


def main(scene="walled"):
    import oracle_py
    from conftest import load_scene

    sc = load_scene(scene)
    if sc.desc.n_free_tris or sc.desc.n_meshes:
        raise SystemExit("the floor is defined for the sphere-only kernel")
    w, h = int(sc.info.width), int(sc.info.height)
    tiles = [(x, y, 1, 1) for y in range(0, h, 16) for x in range(0, w, 16)]
    oracle_py.mix_counts(reset=True)
    _, c = oracle_py.render(sc, tiles, 0, 16, accum=oracle_py.ACCUM_FORWARD, counts=True)
    m = oracle_py.mix_counts(reset=True)
    n = c["samples"]
    per = {"segments": c["segments"] / n, "hits": c["hits"] / n, "draws": m["draws"] / n,
           "diff": m["diff"] / n, "diffspec": (m["diffspec_diff"] + m["diffspec_spec"]) / n,
           "spec": m["spec"] / n, "dielectric": m["dielectric"] / n, "rr_draws": m["rr_draws"] / n,
           "sphere_disc_positive": m["sphere_disc_positive"] / n}
    n_sph = int(sc.desc.n_spheres)
    parts = {
        "sample": OPS["sample"],
        "draws": OPS["draw"] * per["draws"],
        "segments": OPS["segment"] * per["segments"],
        "sphere_discriminants": OPS["sphere_disc"] * n_sph * per["segments"],
        "sphere_roots": OPS["sphere_roots"] * per["sphere_disc_positive"],
        "hit_segments": OPS["hit_segment"] * per["hits"],
        "hits": OPS["hit"] * per["hits"],
        "diffuse": OPS["diff"] * (per["diff"] + m["diffspec_diff"] / n),
        "dielectric": OPS["dielectric"] * per["dielectric"],
        "diffspec_seed": OPS["diffspec_seed"] * per["diffspec"],
        "russian_roulette": OPS["rr"] * per["rr_draws"],
    }
    total = sum(parts.values())
    out = {"scene": scene, "lane_ops_per_sample": round(total, 1),
           "parts": {k: round(v, 1) for k, v in parts.items()},
           "events_per_sample": {k: round(v, 4) for k, v in per.items()}, "spheres": n_sph, "ops": OPS,
           "grid": f"every 16th pixel of {w}x{h}, 16 spp ({n} samples), oracle forward order",
           "note": "the arithmetic bit-exactness fixes (tools/min_insts.py); bench.py divides it by "
                   "64 x SQ_INSTS_VALU per sample (lane-slots issued)"}
    path = os.path.join(ROOT, "profiles", f"min_insts_{scene}.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
