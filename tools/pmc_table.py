"""Summarise rocprofv3 counter-collection CSVs: per kernel (name filter),
the mean over dispatches of each counter, plus per-wave ratios.

    python tools/pmc_table.py DIR [DIR ...] [--kernel env_kernel]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def load(d, kfilter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return None
    per = defaultdict(lambda: defaultdict(float))
    for row in csv.DictReader(open(f[0])):
        if kfilter not in row["Kernel_Name"]:
            continue
        per[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
    if not per:
        return None
    names = sorted({n for v in per.values() for n in v})
    return {n: sum(v.get(n, 0.0) for v in per.values()) / len(per) for n in names}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="env_kernel")
    a = ap.parse_args()
    for d in a.dirs:
        m = load(d, a.kernel)
        if m is None:
            print(d, "no data")
            continue
        w = m.get("SQ_WAVES", 0) or 1
        print(os.path.basename(d.rstrip("/")), " ".join(f"{k.replace('SQ_', '')}={v / w:.0f}/wave" if k != "SQ_WAVES"
                                                         else f"waves={v:.0f}" for k, v in m.items()))


if __name__ == "__main__":
    main()
