"""Summarises tools/gpu_lds_ab.sh (the round-4 ★n2 A/B) into one JSON document: per scene the
Msamples/s of every variant (best of the interleaved rounds, tools/variant_bench.py, images
checked identical), and on a380 each variant's counters per 40-spp launch (the last queue-kernel
dispatch of its rocprofv3 passes): TD / TA busy fraction, vector-memory and LDS wave-instructions
per sample, VALU per sample, wave cycles waiting.
Usage: python tools/lds_ab_summary.py gpurun_out/r4_lds > profiles/r4_lds_ab.json"""
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import counters  # noqa: E402

SAMPLES = 1200 * 600 * 40  # one variant_bench launch


def main(src):
    out = {"source": src, "scenes": {}, "a380_counters": {}}
    for f in sorted(os.listdir(src)):
        m = re.match(r"ab_(\w+)\.log$", f)
        if not m:
            continue
        rows, same = {}, {}
        for line in open(os.path.join(src, f)):
            if line.startswith("{"):
                d = json.loads(line)
                rows[d["variant"]] = d["best"]
            mm = re.match(r"(\S+): identical to (\S+): (\w+)", line)
            if mm:
                same[mm.group(1)] = mm.group(3) == "True"
        out["scenes"][m.group(1)] = {v: {"Msamples_s": r, "bit_identical": same.get(v)} for v, r in rows.items()}
    variants = None
    log = [f for f in os.listdir(src) if f.startswith("tatd_") and f.endswith(".log")]
    for f in sorted(log, key=lambda x: int(re.findall(r"\d+", x)[0])):
        i = re.findall(r"\d+", f)[0]
        name = None
        for line in open(os.path.join(src, f)):
            mm = re.match(r"(\S+): identical", line)
            if mm:
                name = mm.group(1)
        d = {}
        for part in ("tatd", "sq"):
            p = os.path.join(src, f"{part}_{i}", "run_counter_collection.csv")
            if not os.path.exists(p):
                continue
            per, _ = counters(p, kernels=("queue_kernel",))
            if per:
                d.update(list(per.values())[-1])
        if not d or not name:
            continue
        r = {}
        if d.get("GRBM_GUI_ACTIVE"):
            cyc = d["GRBM_GUI_ACTIVE"] / 8
            r["td_busy"] = round(d.get("TD_TD_BUSY_sum", 0) / 256 / cyc, 4)
            r["ta_busy"] = round(d.get("TA_TA_BUSY_sum", 0) / 256 / cyc, 4)
        for k, n in (("SQ_INSTS_VMEM_RD", "vmem_rd_per_sample"), ("SQ_INSTS_LDS", "lds_per_sample"),
                     ("SQ_INSTS_VALU", "valu_per_sample")):
            if k in d:
                r[n] = round(d[k] / SAMPLES, 3)
        if d.get("SQ_WAVE_CYCLES"):
            r["wait_frac"] = round(d.get("SQ_WAIT_ANY", 0) / d["SQ_WAVE_CYCLES"], 4)
        out["a380_counters"][name] = r
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
