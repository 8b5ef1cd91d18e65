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


def bench_line(path):
    if os.path.exists(path):
        for l in open(path):
            if l.startswith("{"):
                return json.loads(l)
    return {}


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
    cnt = {}
    for part, title in (("fetch", "HBM read bytes (FETCH_SIZE, own pass)"), ("sq", "SQ counters (own pass)"),
                        ("sq2", "SQ lane utilisation (own pass)"), ("tcc", "L2 hits / misses (TCC, own pass)"),
                        ("tatd", "Vector-memory units busy (TA / TD, own pass)")):
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
        d = list(per.values())[-1]  # the last trace dispatch
        cfg = bench_line(os.path.join(src, f"bench_{part}.log"))
        if cfg:
            cnt.setdefault("scene", cfg.get("metric", "").split(" on ")[-1].replace(".yml", ""))
            cnt.setdefault("samples_per_launch", cfg.get("launch", {}).get("samples_per_launch", 0))
        if "FETCH_SIZE" in d:
            cnt["hbm_read_bytes_per_launch"] = int(2 * d["FETCH_SIZE"] * 1024)
            lines.append(f"\nLast dispatch: FETCH_SIZE {d['FETCH_SIZE']:.1f} KB -> x2 (gfx950 correction) = "
                         f"{2 * d['FETCH_SIZE'] / 1024:.2f} MB read from HBM per launch.")
        if "SQ_INSTS_VALU" in d:
            cnt["valu_insts_per_launch"] = d["SQ_INSTS_VALU"]
        if "SQ_INSTS_VMEM_RD" in d:
            cnt["vmem_rd_per_launch"] = d["SQ_INSTS_VMEM_RD"]
        if "SQ_THREAD_CYCLES_VALU" in d and d.get("SQ_ACTIVE_INST_VALU"):
            cnt["valu_lane_util"] = round(d["SQ_THREAD_CYCLES_VALU"] / (64 * d["SQ_ACTIVE_INST_VALU"]), 4)
            lines.append(f"\nLast dispatch: VALU lane utilisation = THREAD_CYCLES_VALU / (64 x ACTIVE_INST_VALU) = "
                         f"{cnt['valu_lane_util']:.1%}.")
        if "SQ_WAVE_CYCLES" in d:
            wc = d["SQ_WAVE_CYCLES"]
            cnt["wait_any_frac"] = round(d.get("SQ_WAIT_ANY", 0) / wc, 4)
            cnt["issue_frac"] = round(d.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4)
            cnt["issue_stall_frac"] = round(d.get("SQ_WAIT_INST_ANY", 0) / wc, 4)
            lines.append(f"\nLast dispatch: wait-any {cnt['wait_any_frac']:.1%}, issuing {cnt['issue_frac']:.1%}, "
                         f"issue-stall {cnt['issue_stall_frac']:.1%} of wave cycles.")
        if "TCC_HIT_sum" in d:
            req = d["TCC_HIT_sum"] + d.get("TCC_MISS_sum", 0)
            cnt["l2_bytes_per_launch"] = int(128 * req)
            cnt["l2_hit_rate"] = round(d["TCC_HIT_sum"] / max(req, 1), 4)
            lines.append(f"\nLast dispatch: L2 hit rate {cnt['l2_hit_rate']:.1%}, {req:.4g} requests "
                         f"(x 128 B = {128 * req / 1e9:.3f} GB).")
        if "TD_TD_BUSY_sum" in d and d.get("GRBM_GUI_ACTIVE"):
            # per-instance busy cycles (one TA / TD per CU) over the kernel's cycles per XCD
            # (rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs, MI355X_MICROARCH.md)
            cyc = d["GRBM_GUI_ACTIVE"] / 8
            cnt["td_busy_frac"] = round(d["TD_TD_BUSY_sum"] / 256 / cyc, 4)
            cnt["ta_busy_frac"] = round(d.get("TA_TA_BUSY_sum", 0) / 256 / cyc, 4)
            lines.append(f"\nLast dispatch: texture data (TD) busy {cnt['td_busy_frac']:.1%}, texture address (TA) "
                         f"busy {cnt['ta_busy_frac']:.1%} of the kernel's cycles (per-CU unit, 256 CUs; "
                         f"GRBM_GUI_ACTIVE / 8 XCDs).")
        lines.append("")
    if cnt:
        bid = os.path.join(src, "build_id")
        cnt["build_id"] = open(bid).read().strip() if os.path.exists(bid) else None
        cnt["note"] = ("rocprofv3 --pmc, one counter group per pass, last trace dispatch of the queue kernel; "
                       "FETCH_SIZE x2 per MI355X_MICROARCH.md; build_id = rt_amd.abi.kernel_build_id() of the "
                       "profiled library")
        json.dump(cnt, open(os.path.join(dst, f"{tag}_counters.json"), "w"), indent=1)
    out = os.path.join(dst, f"{tag}_summary.md")
    open(out, "w").write("\n".join(lines) + "\n")
    print(open(out).read())


if __name__ == "__main__":
    main(sys.argv[1])
