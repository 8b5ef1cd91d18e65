"""Sums rocprofv3 --pmc counters over the dispatches of kernels matching a pattern.
Usage: python tools/pmc_sum.py <counter_collection.csv | dir> [kernel-regex] [--per N]
--per N divides every sum by N (e.g. the samples the run traced)."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def main():
    args = [a for a in sys.argv[1:]]
    per = 1.0
    if "--per" in args:
        i = args.index("--per")
        per = float(args[i + 1])
        del args[i:i + 2]
    path = args[0]
    pat = re.compile(args[1] if len(args) > 1 else "queue_kernel")
    if os.path.isdir(path):
        files = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    else:
        files = [path]
    sums = defaultdict(float)
    disp = set()
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if not pat.search(row.get("Kernel_Name", "")):
                    continue
                disp.add((f, row.get("Dispatch_Id")))
                sums[row["Counter_Name"]] += float(row["Counter_Value"])
    print(f"dispatches: {len(disp)}")
    for k in sorted(sums):
        print(f"{k}: {sums[k] / per:.4g}")


if __name__ == "__main__":
    main()
