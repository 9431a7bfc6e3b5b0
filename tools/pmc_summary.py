"""Median per-dispatch PMC counters of one kernel from rocprofv3 CSVs.

    python tools/pmc_summary.py <dir with p*/run_counter_collection.csv> [kernel substring]
"""
import collections, csv, glob, statistics, sys
root = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "env_kernel"
out = {}
for p in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # dispatch -> counter -> sum
    for r in csv.DictReader(open(p)):
        if name in r["Kernel_Name"]:
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    cols = collections.defaultdict(list)
    for d in per.values():
        for k, v in d.items():
            cols[k].append(v)
    for k, v in cols.items():
        out[k] = statistics.median(v)
waves = out.get("SQ_WAVES", 1.0)
print(f"kernel ~ {name}: median per dispatch")
for k in sorted(out):
    print(f"{k:26s} {out[k]:16.0f}   per-wave {out[k]/waves:12.1f}")
