"""Write profiles/traffic_<config>.json (bench.py roofline.traffic) from a
tools/prof_config.py summary.json: HBM bytes per timed step summed over the
step's kernels (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md HBM section),
plus the per-kernel split and the mean kernel durations they were taken with.

    python tools/traffic_from_summary.py gpurun_out/r3_prof/c4/summary.json [--dst profiles/r3/prof/c4]
"""
import argparse
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("summary")
    ap.add_argument("--dst", default=None, help="also copy the summary, bench line and kernel stats here")
    args = ap.parse_args()
    s = json.load(open(args.summary))
    ks = {k: v for k, v in s["kernels"].items() if "random_actions" not in k}
    total = sum(v.get("hbm_bytes", 0) for v in ks.values())
    out = {
        "config": s["config"],
        "warmup": s["warmup"],
        "steps": s["steps"],
        "hbm_bytes_per_launch": total,
        "per_kernel": {k: {"hbm_bytes": v.get("hbm_bytes"), "read": v.get("hbm_read_bytes"),
                           "write": v.get("hbm_write_bytes"), "mean_us": v["mean_us"],
                           "dispatches_per_step": v.get("dispatches_per_step", 1),
                           "per_step_us": v.get("per_step_us", v["mean_us"])} for k, v in ks.items()},
        "step_mean_us": round(sum(v.get("per_step_us", v["mean_us"]) for v in ks.values()), 3),
        "source": f"tools/prof_config.py --config {s['config']} --steps {s['steps']} --warmup {s['warmup']}: "
                  "separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, the timed region's dispatches of each "
                  "per-step kernel (bytes per step), FETCH_SIZE x2 (gfx950 counts half of each 128-B request)",
    }
    dst = os.path.join(ROOT, "profiles", f"traffic_{s['config']}.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(dst, total)
    if args.dst:
        src = os.path.dirname(args.summary)
        os.makedirs(args.dst, exist_ok=True)
        shutil.copy(args.summary, args.dst)
        for name in ("bench.json",):
            if os.path.exists(os.path.join(src, name)):
                shutil.copy(os.path.join(src, name), args.dst)
        ks_csv = os.path.join(src, "trace", "run_kernel_stats.csv")
        if os.path.exists(ks_csv):
            shutil.copy(ks_csv, os.path.join(args.dst, "kernel_stats.csv"))


if __name__ == "__main__":
    sys.exit(main())
