"""Why the CPU baseline's repeated calls differ (bench.py cpu_baseline; round 5 triangles
35 / 112 / 33 Msamples/s at the same CPU-seconds per call): the same oracle call, repeated,
floating over every host CPU as bench.py runs it vs pinned to the least-busy physical cores
(one hardware thread per core, cores picked from /proc/stat just before each call).
Per call it records the rate, the effective cores and the host's busy fraction.
Usage: python tools/cpu_baseline_probe.py [--scene triangles] [--spp 200] [--reps 4]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def cpu_times():
    out = {}
    for line in open("/proc/stat"):
        if line.startswith("cpu") and line[3].isdigit():
            f = line.split()
            v = list(map(int, f[1:]))
            out[int(f[0][3:])] = (sum(v) - v[3] - v[4], sum(v))  # busy (not idle/iowait), total
    return out


def busy_fracs(window=0.5):
    a = cpu_times()
    time.sleep(window)
    b = cpu_times()
    return {c: (b[c][0] - a[c][0]) / max(b[c][1] - a[c][1], 1) for c in a if c in b}


def cores():
    """physical core -> its hardware threads, from sysfs."""
    groups = {}
    for c in os.sched_getaffinity(0):
        try:
            sib = open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip()
        except OSError:
            sib = str(c)
        groups.setdefault(sib, []).append(c)
    return list(groups.values())


def pick(n, busy):
    """n least-busy physical cores (busy of all their hardware threads), one thread each."""
    cs = sorted(cores(), key=lambda g: sum(busy.get(c, 1.0) for c in g))
    return [min(g) for g in cs[:n]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="triangles")
    ap.add_argument("--spp", type=int, default=200)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--threads", type=int, default=16)
    args = ap.parse_args()
    import bench
    import oracle_py

    _, loaded = bench.load(args.scene)
    w, h = int(loaded.info.width), int(loaded.info.height)
    tiles = [(0, 0, w, h)]
    allowed = os.sched_getaffinity(0)
    oracle_py.render(loaded, tiles, 0, 0, threads=args.threads)
    oracle_py.render(loaded, tiles, 0, args.spp, threads=args.threads)
    rows = []
    for rep in range(args.reps):
        for mode in ("float", "pinned"):
            busy = busy_fracs()
            host_busy = sum(busy.values()) / max(len(busy), 1)
            cpus = pick(args.threads, busy) if mode == "pinned" else sorted(allowed)
            os.sched_setaffinity(0, cpus)
            c0, t0 = os.times(), time.perf_counter()
            oracle_py.render(loaded, tiles, 0, args.spp, threads=args.threads)
            t1, c1 = time.perf_counter(), os.times()
            os.sched_setaffinity(0, allowed)
            cpu = (c1.user - c0.user) + (c1.system - c0.system)
            row = {"rep": rep, "mode": mode, "Msamples_s": round(w * h * args.spp / (t1 - t0) / 1e6, 3),
                   "wall_s": round(t1 - t0, 3), "effective_cores": round(cpu / (t1 - t0), 2),
                   "host_busy_before": round(host_busy, 3),
                   "cpus": cpus if mode == "pinned" else f"{len(cpus)} allowed"}
            rows.append(row)
            print(json.dumps(row), flush=True)
    for mode in ("float", "pinned"):
        v = sorted(r["Msamples_s"] for r in rows if r["mode"] == mode)
        med = v[len(v) // 2]
        print(json.dumps({"mode": mode, "median": med, "min": v[0], "max": v[-1],
                          "spread": round((v[-1] - v[0]) / med, 4)}), flush=True)


if __name__ == "__main__":
    main()
