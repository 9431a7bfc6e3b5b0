"""Copy a gpu_profile.sh run into profiles/ and derive the bench's HBM traffic.

    python tools/make_traffic.py gpurun_out/prof_<tag> profiles/r1/<tag> [--config c2]

Writes <dst>/kernel_stats.csv (rocprofv3 --kernel-trace --stats of the default
bench command), <dst>/pmc_<group>.csv (env-kernel rows of each separate --pmc
pass), <dst>/summary.txt, and profiles/traffic_<config>.json, whose
hbm_bytes_per_launch bench.py reports as roofline.traffic.  HBM bytes follow
MI355X_MICROARCH.md: FETCH_SIZE (KiB) counts half of each 128-B request on
gfx950 (x2), WRITE_SIZE (KiB) as is.
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--config", default="c2")
    args = ap.parse_args()
    os.makedirs(args.dst, exist_ok=True)
    shutil.copy(os.path.join(args.src, "trace", "run_kernel_stats.csv"),
                os.path.join(args.dst, "kernel_stats.csv"))
    avg = {}
    kname = None
    for p in sorted(glob.glob(os.path.join(args.src, "p*", "run_counter_collection.csv"))):
        grp = os.path.basename(os.path.dirname(p))
        rows = [r for r in csv.DictReader(open(p)) if "env_kernel" in r["Kernel_Name"]]
        if not rows:
            continue
        kname = rows[0]["Kernel_Name"]
        with open(os.path.join(args.dst, f"{grp}.csv"), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(rows)
        agg = collections.defaultdict(list)
        for r in rows:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            avg[k] = sum(v) / len(v)
    waves = avg.get("SQ_WAVES", 1.0)
    with open(os.path.join(args.dst, "summary.txt"), "w") as f:
        f.write(f"kernel: {kname}\nper-dispatch averages over the profiled launches\n")
        for k in sorted(avg):
            f.write(f"{k:30s} {avg[k]:16.1f}   per-wave {avg[k] / waves:10.1f}\n")
    import bench
    c = bench.CONFIGS[args.config]
    bpe = bench.algorithmic_bytes_per_env_step(c["numrobot"], c["sensor_config"]["range"], 2)
    fetch, write = avg.get("FETCH_SIZE"), avg.get("WRITE_SIZE")
    hbm = None if fetch is None or write is None else int(round((2 * fetch + write) * 1024))
    out = {
        "config": args.config,
        "kernel": kname,
        "source": f"{args.dst}/pmc_*.csv (rocprofv3 --pmc, separate passes, "
                  "tools/gpu_pmc_traffic.sh)",
        "fetch_size_kb_per_launch": fetch,
        "write_size_kb_per_launch": write,
        "correction": "MI355X_MICROARCH.md HBM section: FETCH_SIZE reads 1/2 of the bytes of "
                      "128-B requests on gfx950 -> x2; WRITE_SIZE taken as is",
        "hbm_bytes_per_launch": hbm,
        "alg_bytes_per_launch": bpe * c["envs"],
        "tcc_hit_rate": (round(avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"]), 3)
                         if "TCC_HIT_sum" in avg else None),
        "per_wave": {k: round(v / waves, 1) for k, v in avg.items() if k.startswith("SQ_")},
    }
    with open(os.path.join(ROOT, "profiles", f"traffic_{args.config}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
