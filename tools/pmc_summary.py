"""Average per-dispatch PMC counters of the env kernel from rocprofv3 CSVs."""
import collections, csv, glob, sys
root = sys.argv[1]
waves = None
out = {}
for p in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(p)):
        if "env_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        out[k] = sum(v) / len(v)
waves = out.get("SQ_WAVES", 1.0)
for k in sorted(out):
    print(f"{k:26s} {out[k]:16.0f}   per-wave {out[k]/waves:12.1f}")
