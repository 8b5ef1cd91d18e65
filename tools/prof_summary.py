"""Summarises a tools/run_profiles.sh output directory into profiles/<tag>_summary.md and
copies the raw rocprofv3 CSVs that back it.  Usage: python tools/prof_summary.py <tag>"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path, kernels=("queue_kernel", "trace_kernel")):
    rows = list(csv.DictReader(open(path)))
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in rows:
        k = r["Kernel_Name"]
        if any(n in k for n in kernels) and "trace_kernel<true" not in k:
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
    return per, names


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    lines = [f"# rocprofv3 summary — {tag}", ""]
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
        lines += ["## Kernel trace (`rocprofv3 --kernel-trace --stats`)", "", "| kernel | calls | avg ms | min ms | max ms | % |",
                  "|---|---|---|---|---|---|"]
        for r in csv.DictReader(open(stats)):
            lines.append(f"| `{r['Name'][:70]}` | {r['Calls']} | {float(r['AverageNs'])/1e6:.3f} | "
                         f"{float(r['MinNs'])/1e6:.3f} | {float(r['MaxNs'])/1e6:.3f} | {r['Percentage']} |")
        lines.append("")
    bench = os.path.join(src, "bench_trace.log")
    if os.path.exists(bench):
        for l in open(bench):
            if l.startswith("{"):
                d = json.loads(l)
                lines += ["## bench.py line (under the profiler)", "", "```", l.strip(), "```", ""]
    valu = {}
    for part, title in (("fetch", "HBM read bytes (FETCH_SIZE, own pass)"), ("sq", "SQ counters (own pass)"),
                        ("sq2", "SQ lane utilisation (own pass)")):
        p = os.path.join(src, part, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        shutil.copy(p, os.path.join(dst, f"{tag}_{part}_counters.csv"))
        per, names = counters(p)
        if not per:
            continue
        keys = sorted({k for d in per.values() for k in d})
        lines += [f"## {title}", "", "| dispatch | " + " | ".join(keys) + " |", "|---" * (len(keys) + 1) + "|"]
        for did, d in sorted(per.items(), key=lambda x: int(x[0])):
            lines.append(f"| {did} | " + " | ".join(f"{d[k]:.4g}" for k in keys) + " |")
        d = list(per.values())[-1]
        if "FETCH_SIZE" in d:
            lines.append(f"\nLast dispatch: FETCH_SIZE {d['FETCH_SIZE']:.1f} KB -> x2 (gfx950 correction) = "
                         f"{2 * d['FETCH_SIZE'] / 1024:.2f} MB read from HBM per launch.")
            bl = os.path.join(src, "bench_fetch.log")
            cfg = {}
            if os.path.exists(bl):
                for l in open(bl):
                    if l.startswith("{"):
                        cfg = json.loads(l)
            scene = cfg.get("metric", "").split(" on ")[-1].replace(".yml", "") if cfg else None
            spl = cfg.get("launch", {}).get("samples_per_launch", 0)
            json.dump({"scene": scene, "samples_per_launch": spl,
                       "hbm_read_bytes_per_launch": int(2 * d["FETCH_SIZE"] * 1024),
                       "note": "rocprofv3 --pmc FETCH_SIZE, own pass, last trace dispatch, x2 per "
                               "MI355X_MICROARCH.md HBM section"},
                      open(os.path.join(dst, f"{tag}_fetch.json"), "w"), indent=1)
        if "SQ_INSTS_VALU" in d:
            valu["valu_insts_per_launch"] = d["SQ_INSTS_VALU"]
        if "SQ_THREAD_CYCLES_VALU" in d and d.get("SQ_ACTIVE_INST_VALU"):
            valu["valu_lane_util"] = round(d["SQ_THREAD_CYCLES_VALU"] / (64 * d["SQ_ACTIVE_INST_VALU"]), 4)
        if "SQ_WAVE_CYCLES" in d:
            wc = d["SQ_WAVE_CYCLES"]
            lines.append(f"\nLast dispatch: wait-any {d.get('SQ_WAIT_ANY', 0) / wc:.1%}, issuing {d.get('SQ_ACTIVE_INST_ANY', 0) / wc:.1%}, "
                         f"issue-stall {d.get('SQ_WAIT_INST_ANY', 0) / wc:.1%} of wave cycles.")
        if "SQ_THREAD_CYCLES_VALU" in d and d.get("SQ_ACTIVE_INST_VALU"):
            lines.append(f"\nLast dispatch: VALU lane utilisation = THREAD_CYCLES_VALU / (64 x ACTIVE_INST_VALU) = "
                         f"{d['SQ_THREAD_CYCLES_VALU'] / (64 * d['SQ_ACTIVE_INST_VALU']):.1%}.")
        lines.append("")
    if "valu_insts_per_launch" in valu:
        bl = os.path.join(src, "bench_sq.log")
        cfg = {}
        if os.path.exists(bl):
            for l in open(bl):
                if l.startswith("{"):
                    cfg = json.loads(l)
        valu.update({"scene": cfg.get("metric", "").split(" on ")[-1].replace(".yml", "") if cfg else None,
                     "samples_per_launch": cfg.get("launch", {}).get("samples_per_launch", 0),
                     "note": "rocprofv3 --pmc SQ_INSTS_VALU (wave-level VALU instructions, all XCDs) and "
                             "THREAD_CYCLES_VALU / (64 x ACTIVE_INST_VALU), own passes, last trace dispatch"})
        json.dump(valu, open(os.path.join(dst, f"{tag}_valu.json"), "w"), indent=1)
    out = os.path.join(dst, f"{tag}_summary.md")
    open(out, "w").write("\n".join(lines) + "\n")
    print(open(out).read())


if __name__ == "__main__":
    main(sys.argv[1])
