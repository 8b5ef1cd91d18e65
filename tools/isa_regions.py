"""Static instruction accounting of one trace kernel by source region.

Disassembles the kernel from a line-table build of csrc/kernel/trace.hip (`make -C
gpu-ray_trace-rust_amd isa-lines`: the same code, byte for byte, as the shipped library — the tool
checks it), symbolizes every instruction with its inline stack (llvm-symbolizer --inlining) and
assigns it to a region of the path (discriminants, roots, in_return_leaf, shading branches,
path starts, queue, ...).  Prints, per region, the instruction counts by class (VALU, SALU, VMEM,
SMEM, LDS, branch/wait), and — with --samples, a CSV of PC samples (address, count) from
rocprofv3 --pc-sampling — the sampled share of each region.

Usage: python tools/isa_regions.py [--kernel 'queue_kernelILb0ELb0ELb1ELb0EE'] [--samples pcs.csv] [--json out]
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gpu-ray_trace-rust_amd")
LLVM = "/opt/rocm/lib/llvm/bin"

# (region, pattern): matched against the instruction's inline stack written outermost first,
# frames joined by ">" ("queue_kernel>segment>closest_small>sphere_disc>dot"); the first rule
# that matches names the region.
RULES = [
    ("closest: discriminants", r">closest_small<[^>]*>.*sphere_disc"),
    ("closest: roots", r">closest_small<[^>]*>.*sphere_roots"),
    ("closest: in_return_leaf", r">closest_small<[^>]*>.*in_return_leaf"),
    ("closest: ray axes + root slab", r">closest_small<[^>]*>.*(ray_axes|entry_exit)"),
    ("closest: fallback traversal", r">closest_small<[^>]*>.*stack_search"),
    ("closest: selection + loop", r">closest_small"),
    ("shade: libm sin/cos (diffuse angle)", r">shade<.*rt_sincosf"),
    ("shade: libm powf(c, 5) (Fresnel)", r">shade<.*rt_powf5"),
    ("shade: rng draws", r">shade<.*rt_rng_"),
    ("shade: diffuse continue", r">shade<.*diff_vec"),
    ("shade: refraction", r">shade<.*refract_vec"),
    ("shade: hit info, emission, RR, mirror, throughput", r">shade<"),
    ("segment: normalize", r">segment<.*normalize"),
    ("path starts (camera ray, stream start)", r"make_start|camera_ray|camera_base_dir|start_path|split_item"),
    ("setup: LDS tables", r"fill_lds_spheres"),
]
CLASSES = [("VALU", r"^v_"), ("SALU", r"^s_(?!load|buffer_load|waitcnt|cbranch|branch|barrier|nop|endpgm|setprio|sleep)"),
           ("VMEM", r"^(global_|buffer_|flat_|scratch_)"), ("SMEM", r"^s_(load|buffer_load)"), ("LDS", r"^ds_"),
           ("branch/wait", r"^s_(waitcnt|cbranch|branch|barrier|nop|endpgm|setprio|sleep)")]


def code_object(lib):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_device_code import _gfx950_object

    return _gfx950_object(lib)


def kernel_text(elf_path, kernel):
    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", elf_path], capture_output=True,
                         text=True, check=True).stdout
    insts, on = [], False
    for line in out.splitlines():
        if line.endswith(">:") and "<" in line:
            on = kernel in line
            continue
        if not on:
            continue
        m = re.match(r"\s+(\S+)(.*?)//\s*([0-9A-Fa-f]+):", line)
        if m:
            insts.append((int(m.group(3), 16), m.group(1), m.group(2).strip()))
    return insts


def symbolize(elf_path, addrs):
    r = subprocess.run([f"{LLVM}/llvm-symbolizer", "--inlining", "--demangle", "--output-style=JSON",
                        f"--obj={elf_path}"], input="\n".join(hex(a) for a in addrs), capture_output=True, text=True,
                       check=True)
    stacks = []
    for line in r.stdout.splitlines():
        d = json.loads(line)
        stacks.append([(f.get("FunctionName", ""), f.get("Line", 0)) for f in d.get("Symbol", [])])
    return stacks


def region_of(stack):
    chain = ">" + ">".join(re.sub(r"^rtd::", "", fn) for fn, _ in reversed(stack))  # outermost first
    for name, pat in RULES:
        if re.search(pat, chain):
            return name
    return "queue: regen, grabs, loop, radiance store"


def klass(mn):
    for c, pat in CLASSES:
        if re.match(pat, mn):
            return c
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="queue_kernelILb0ELb0ELb1ELb0EE")
    ap.add_argument("--lines-elf", default=os.path.join(PKG, "build", "trace_lines.elf"))
    ap.add_argument("--lib", default=os.path.join(PKG, "lib", "librt_amd.so"))
    ap.add_argument("--samples", default=None, help="CSV of pc,count (absolute code-object addresses)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    insts = kernel_text(a.lines_elf, a.kernel)
    # the line-table build must be the shipped code, byte for byte
    shipped = os.path.join(PKG, "build", "shipped_gfx950.elf")
    open(shipped, "wb").write(code_object(a.lib))
    ref = kernel_text(shipped, a.kernel)
    same = [(i[1], i[2]) for i in insts] == [(i[1], i[2]) for i in ref]
    stacks = symbolize(a.lines_elf, [i[0] for i in insts])
    table = collections.OrderedDict()
    per_pc = {}
    for (pc, mn, _ops), st in zip(insts, stacks):
        reg = region_of(st)
        per_pc[pc] = reg
        row = table.setdefault(reg, collections.Counter())
        row[klass(mn)] += 1
        row["all"] += 1
    res = {"kernel": a.kernel, "instructions": len(insts), "same_as_shipped": same,
           "static": {k: dict(v) for k, v in table.items()}}
    if a.samples:
        samp = collections.Counter()
        total = 0
        for line in open(a.samples):
            p = line.strip().split(",")
            if len(p) < 2 or not p[1].strip().isdigit():
                continue
            pc, n = int(p[0], 0), int(p[1])
            total += n
            samp[per_pc.get(pc, "outside the kernel")] += n
        res["samples"] = {k: {"n": v, "share": round(v / total, 4)} for k, v in samp.most_common()}
    print(json.dumps(res, indent=1))
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
