"""Walled instruction accounting: where the sphere-only queue kernel's VALU issue
goes, region by region, reconciled with the SQ_INSTS_VALU counter of the shipped build.

Dynamic side: the RT_REGION_COUNT diagnostic library (`make -C gpu-ray_trace-rust_amd diag` ->
lib/variants/librt_diag_regions.so; csrc/kernel/diag.h RC_*) counts, per launch, how many times a
wave runs through each region of the path (the first active lane counts: one count per
wave-instruction stream).  Static side: tools/isa_regions.py's per-instruction region
attribution of the SHIPPED kernel's ISA (the line-table build, byte-identical), grouped into the
hot code of each region; VALU instructions per execution = the region's hot VALU instructions /
its static copies (loop bodies unrolled or duplicated by the compiler).  Issued VALU per region
= executions x VALU per execution.

Usage:
  on the GPU box:  python tools/walled_accounting.py --gpu > profiles/<tag>_walled_regions.json
  here:            python tools/walled_accounting.py --table profiles/<tag>_walled_regions.json
                       [--sq-valu N]   (SQ_INSTS_VALU per launch of the product build, same launch)
"""
import argparse
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gpu-ray_trace-rust_amd")
RC_NAMES = ["iter", "iter_lanes", "regen", "batch", "roots", "slab", "fallback", "fb_nodes", "fb_leaves",
            "shade_hit", "seed", "rr", "spec", "dielectric", "diff", "atten_div", "store", "cube", "pow_slow", "roots_useful", "roots_front"]

CHILD = r"""
import os, sys
sys.path.insert(0, os.path.join(%(root)r, "gpu-ray_trace-rust_amd"))
import torch  # noqa: F401
from rt_amd import abi, render, scheme
lib = abi.load_library(os.path.join(%(root)r, "gpu-ray_trace-rust_amd", "lib", "variants", "librt_diag_regions.so"))
sch = scheme.load_json(os.path.join(%(root)r, "tests", "golden", "scenes", "walled.json"))
loaded = scheme.load(sch, lib=lib)
with render.Context(loaded, lib=lib) as c:
    c.render(None, 0, %(spp)d, want_output=False)
    print("LAUNCHES", c.launch_stats()["n_trace_launches"], flush=True)
print("SAMPLES", int(loaded.info.width) * int(loaded.info.height) * %(spp)d, flush=True)
"""


def gpu(spp):
    env = dict(os.environ, RT_DEBUG_LAUNCH="overlap=0")
    r = subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT, "spp": spp}], capture_output=True, text=True,
                       timeout=600, env=env)
    counts, samples, launches = {}, None, None
    for line in r.stdout.splitlines():
        m = re.match(r"RT_RC (\d+) (\d+)", line)
        if m and int(m.group(1)) < len(RC_NAMES):
            counts[RC_NAMES[int(m.group(1))]] = counts.get(RC_NAMES[int(m.group(1))], 0) + int(m.group(2))
        if line.startswith("SAMPLES"):
            samples = int(line.split()[1])
        if line.startswith("LAUNCHES"):
            launches = int(line.split()[1])
    if not counts:
        raise SystemExit(r.stdout[-2000:] + r.stderr[-2000:])
    print(json.dumps({"scene": "walled", "spp": spp, "samples": samples, "launches": launches, "counts": counts}))


def src_line(pattern, start=1):
    """Line number (1-based) of the first trace.hip line at or after `start` containing pattern."""
    for i, line in enumerate(open(os.path.join(PKG, "csrc", "kernel", "trace.hip")), 1):
        if i >= start and pattern in line:
            return i
    raise SystemExit(f"trace.hip: no line with {pattern!r}")


def blocks(elf, kernel):
    """The kernel's basic blocks: [(first pc, [(pc, mnemonic, inline stack)])], split at branch
    targets (llvm-objdump --symbolize-operands labels) and after branches."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_regions as R

    out = subprocess.run([f"{R.LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", "--symbolize-operands", elf],
                         capture_output=True, text=True, check=True).stdout
    insts, labels, on = [], set(), False
    for line in out.splitlines():
        if line.endswith(">:") and "<" in line:
            name = line.split("<", 1)[1]
            if kernel in name:
                on = True
            elif on and name.startswith("L"):
                labels.add(int(line.split()[0], 16))
            elif on:
                on = False
            continue
        if on:
            m = re.match(r"\s+(\S+)(.*?)//\s*([0-9A-Fa-f]+):", line)
            if m:
                insts.append((int(m.group(3), 16), m.group(1), m.group(2)))
    stacks = R.symbolize(elf, [i[0] for i in insts])
    bl, cur = [], None
    for (pc, mn, ops), st in zip(insts, stacks):
        if cur is None or pc in labels:
            cur = (pc, [])
            bl.append(cur)
        cur[1].append((pc, mn, st, ops))
        if mn.startswith(("s_cbranch", "s_branch", "s_endpgm", "s_setpc")):
            cur = None
    return bl, R


def event_of(stack, L):
    """The RC event whose count is an instruction's wave-level execution count (see diag.h), from
    its inline stack (innermost first) and the source anchors L; None: no vote (compiler-made)."""
    ch = [(re.sub(r"[<(].*", "", f).replace("rtd::", "").replace("void ", ""), ln) for f, ln in reversed(stack)]
    names = [f for f, _ in ch]
    lines = dict(ch)
    if not ch or all(ln == 0 for _, ln in ch):
        return None
    has = lambda n: n in names  # noqa: E731
    if has("fill_lds_spheres"):
        return "waves"
    if has("make_start"):
        return "batch"
    if has("closest_small"):
        if has("stack_search"):
            if has("leaf_closest"):
                return "fb_leaves"
            return "fb_nodes" if (has("split_t") or has("fetch_node") or has("sel3")) else "fallback"
        if has("in_return_leaf") or has("fetch_sphere"):
            return "slab"
        if has("entry_exit") or has("ray_axes"):
            return "fallback"  # round 6: the exact slab runs only where the shortcut failed
        # the sphere loop: pairs (lines pair0..pair1: two copies, 6 iterations for 13 spheres) and
        # the remainder (one copy, one iteration); a copy's share of the root computations is
        # taken as its share of the spheres (6/13 per pair copy, 1/13 for the remainder)
        cl = lines.get("closest_small", 0)
        part = "pair" if L["pair0"] <= cl <= L["pair1"] else "rem"
        if has("sphere_disc"):
            return "sphere_" + part
        if has("operator"):  # the take lambda: its first line is the per-sphere ballot
            ln = [l for f, l in ch if f == "operator"][-1]
            return ("sphere_" if ln == L["ballot"] else "roots_") + part
        if has("sphere_roots"):
            return "roots_" + part
        ln = lines.get("closest_small", 0)
        if L["slab0"] <= ln <= L["slab1"]:
            return "slab"
        if L["slab1"] < ln <= L["fb1"]:
            return "fallback"
        return "iter"
    if has("closest"):
        return "dead"  # the general (non-small) traversal: walled always takes closest_small
    if has("shade"):
        if has("cube_emissive"):
            return "cube"
        if has("diff_vec"):
            return "diff"
        if has("rt_powf5_glibc"):
            return "pow_slow"
        if has("refract_vec"):
            return "dielectric"
        if has("div3"):
            return "atten_div"
        ln = lines.get("shade", 0)
        if ln == L["seed"]:
            return "seed"
        if L["rr0"] <= ln <= L["rr1"]:
            return "rr"
        if L["spec0"] <= ln <= L["spec1"]:
            return "spec"
        return "shade_hit"
    if has("segment"):
        return "iter"
    if has("start_path") or has("launch_pixel"):
        return "dead"  # the per-lane start path: walled's camera has no lens, so batched starts
    ln = lines.get("queue_kernel", 0)
    if L["batch0"] <= ln <= L["batch1"]:
        return "batch"
    if L["regen0"] <= ln <= L["regen1"]:
        return "regen"
    if L["dead0"] <= ln <= L["dead1"]:
        return "dead"
    if L["store0"] <= ln <= L["store1"]:
        return "store"
    if ln and ln < L["loop"]:
        return "waves"
    return "iter"


def anchors():
    L = {"ballot": src_line("__ballot(q.thing2 > 0.0f) == 0"),
         "pair0": src_line("const SphDisc qa = sphere_disc(sa, sa.w, r)") - 2,
         "pair1": src_line("const SphDisc qa = sphere_disc(sa, sa.w, r)") + 3,
         "slab0": src_line("RC(RC_SLAB)") - 1, "slab1": src_line("RC(RC_FALLBACK)") - 1,
         "seed": src_line("seed_diff = draw(&p.rng) < m->diffp"),
         "rr0": src_line("russian_roulette_filter"), "rr1": src_line("russian_roulette_filter") + 5,
         "spec0": src_line("RC(RC_SPEC)") - 1, "spec1": src_line("RC(RC_SPEC)") + 1,
         "regen0": src_line("RC(RC_REGEN)") - 1, "batch0": src_line("RC(RC_BATCH)") - 1,
         "loop": src_line("const uint64_t need = __ballot(!have && !done)")}
    L["fb1"] = src_line("if (found) return true;", L["slab1"])
    L["batch1"] = src_line("st_n = 64u - st_pos;", L["batch0"])
    L["dead0"] = src_line("} else if (regen) {", L["regen0"])
    L["regen1"] = L["dead0"] - 1
    L["dead1"] = src_line("if (__ballot(have) == 0) {", L["dead0"]) - 1
    L["store0"] = src_line("if (fin) {", L["dead1"])
    L["store1"] = L["store0"] + 9
    return L


def table(path, sq_valu):
    d = json.load(open(path))
    n = d["counts"]
    elf = os.path.join(PKG, "build", "trace_lines.elf")
    bl, R = blocks(elf, "queue_kernelILb0ELb0ELb1ELb0EE")
    L = anchors()
    # the launch's waves: the grid is the resident workgroups (2 waves each), ~7 per SIMD
    waves = n.get("waves") or d.get("grid_waves") or 256 * 4 * 7
    n_spheres = 13
    cnt = dict(n)
    pairs = n_spheres // 2
    cnt.update(waves=waves, dead=0, cold=0, sphere_pair=pairs * n["iter"], sphere_rem=(n_spheres - 2 * pairs) * n["iter"],
               roots_pair=n["roots"] * pairs / n_spheres, roots_rem=n["roots"] * (n_spheres - 2 * pairs) / n_spheres)
    per_region, per_event, unvoted = {}, {}, 0
    total = 0.0
    prev_ev, prev_falls = None, False
    for pc0, ins in bl:
        votes = {}
        for pc, mn, st, ops in ins:
            # compiler-made instructions (line 0 in the innermost frame: copies, spills, merged
            # tails) do not vote; they run where their block runs
            if mn.startswith("v_") and st and st[0][1] != 0:
                e = event_of(st, L)
                if e:
                    votes[e] = votes.get(e, 0) + 1
        valu = [(pc, mn, st) for pc, mn, st, ops in ins if mn.startswith("v_")]
        falls = not ins[-1][1].startswith(("s_branch", "s_endpgm", "s_setpc"))
        if votes:
            ev = max(votes, key=votes.get)
        elif prev_falls and prev_ev:
            ev = prev_ev  # a block of compiler-made instructions: its fall-through predecessor's event
        else:
            ev = None
        prev_ev, prev_falls = ev, falls
        if not valu:
            continue
        if ev is None and not any(mn.startswith("v_sqrt_f32") for _, mn, _ in valu):
            unvoted += len(valu)
            continue
        if ev is None:
            ev = "cold"  # hipcc's sqrtf behind sqrt_nonneg's guard: its compiler-made copies
        # out-of-line exactness fallbacks (IEEE division, sqrtf's tiny-input scaling): the guarded
        # branches no lane normally takes; counted as not executed
        if any(mn.startswith(("v_div_scale", "v_div_fmas", "v_div_fixup")) for _, mn, _, _ in ins) or \
                (any(mn.startswith(("v_cmp_class", "v_sqrt_f32")) for _, mn, _, _ in ins) and
                 any("0x4f800000" in ops for _, _, _, ops in ins)):
            ev = "cold"
        c = cnt.get(ev, 0)
        for pc, mn, st in valu:
            reg = R.region_of(st)
            per_region.setdefault(reg, [0, 0.0])
            per_region[reg][0] += 1
            per_region[reg][1] += c
        per_event.setdefault(ev, [0, 0.0])
        per_event[ev][0] += len(valu)
        per_event[ev][1] += len(valu) * c
        total += len(valu) * c
    samples = d["samples"]
    out = {"source": os.path.relpath(path, ROOT), "samples": samples, "launches": d.get("launches"),
           "events_per_sample": {k: round(v / samples, 5) for k, v in cnt.items() if k not in ("dead", "cold")},
           "modelled_valu_per_launch": total, "modelled_valu_per_sample": round(total / samples, 3),
           "unvoted_static_valu": unvoted,
           "by_region": {k: {"static_valu": v[0], "valu_per_sample": round(v[1] / samples, 3)}
                         for k, v in sorted(per_region.items(), key=lambda kv: -kv[1][1])},
           "by_event": {k: {"static_valu": v[0], "valu_per_sample": round(v[1] / samples, 3),
                            "executions_per_sample": round(cnt.get(k, 0) / samples, 5)}
                        for k, v in sorted(per_event.items(), key=lambda kv: -kv[1][1])}}
    if sq_valu:
        out["sq_insts_valu_per_sample"] = round(sq_valu / samples, 3)
        out["modelled_over_counter"] = round(total / sq_valu, 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--spp", type=int, default=1000)
    ap.add_argument("--table", default=None)
    ap.add_argument("--sq-valu", type=float, default=None)
    a = ap.parse_args()
    if a.gpu:
        gpu(a.spp)
    if a.table:
        table(a.table, a.sq_valu)
