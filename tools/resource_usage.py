#!/usr/bin/env python3
"""Per-kernel register / scratch / LDS table of the trace library (hipcc's
-Rpass-analysis=kernel-resource-usage remarks, `make isa`).  Usage: tools/resource_usage.py"""
import os
import re
import subprocess
import sys

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu-ray_trace-rust_amd")
KEYS = ("VGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]",
        "LDS Size [bytes/block]")


def main():
    p = subprocess.run(["make", "-s", "-B", "isa"], cwd=PKG, capture_output=True, text=True)
    if p.returncode:
        sys.stderr.write(p.stderr)
        raise SystemExit(p.returncode)
    rows, cur = [], None
    for line in p.stderr.splitlines():
        m = re.search(r"remark:\s+(.*?)(?: \[-Rpass)", line)
        if not m:
            continue
        txt = m.group(1).strip()
        if txt.startswith("Function Name:"):
            name = txt.split(":", 1)[1].strip()
            dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
            cur = {"name": re.sub(r"\(rtd::LaunchArgs\)", "", dem)}
            rows.append(cur)
        elif cur is not None and ":" in txt:
            k, v = txt.split(":", 1)
            if k.strip() in KEYS:
                cur[k.strip()] = v.strip()
    print(f"{'kernel':44s} {'VGPR':>5s} {'vspill':>6s} {'sspill':>6s} {'scratch':>7s} {'waves':>5s} {'LDS':>6s}")
    for r in rows:
        print(f"{r['name'][:44]:44s} {r.get('VGPRs', '?'):>5s} {r.get('VGPRs Spill', '?'):>6s} "
              f"{r.get('SGPRs Spill', '?'):>6s} {r.get('ScratchSize [bytes/lane]', '?'):>7s} "
              f"{r.get('Occupancy [waves/SIMD]', '?'):>5s} {r.get('LDS Size [bytes/block]', '?'):>6s}")


if __name__ == "__main__":
    main()
