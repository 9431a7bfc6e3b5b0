"""Itemise the driver's short bench form (bench.py --steps 20 --warmup 5)
from a rocprofv3 --kernel-trace --hip-trace run:
host wall time of the timed region vs the sum of its kernel durations.

The timed region in the HIP API trace: the last two hipEventRecord calls
(ev0, ev1) bracket the K env-kernel launches; the hipDeviceSynchronize after
ev1 closes it.  Items: host time from ev0's record to the first launch call,
first launch call -> first kernel start (queue-to-start), the gaps between
consecutive kernels, the last kernel's end -> the synchronize's return
(wake-up), and the kernels themselves.

    python3 tools/short_form_trace.py <trace dir> [K]
"""
import csv
import glob
import json
import os
import statistics
import sys


def load(d, name):
    p = glob.glob(os.path.join(d, "**", f"*{name}.csv"), recursive=True)
    with open(p[0]) as f:
        return list(csv.DictReader(f))


def main(d, K=20):
    api = load(d, "hip_api_trace")
    kern = load(d, "kernel_trace")
    t = lambda r, k: int(r[k])  # noqa: E731  (ns)
    api.sort(key=lambda r: t(r, "Start_Timestamp"))
    recs = [r for r in api if r["Function"] == "hipEventRecord"]
    ev0, ev1 = recs[-2], recs[-1]
    launches = [r for r in api if r["Function"] == "hipLaunchKernel" and
                t(ev0, "End_Timestamp") <= t(r, "Start_Timestamp") <= t(ev1, "Start_Timestamp")]
    syncs = [r for r in api if r["Function"] == "hipDeviceSynchronize" and
             t(r, "Start_Timestamp") >= t(ev1, "End_Timestamp")]
    sync = syncs[0]
    env = sorted([r for r in kern if "env_kernel" in r["Kernel_Name"]], key=lambda r: t(r, "Start_Timestamp"))
    timed = env[-K:]
    assert len(launches) == K, len(launches)
    durs = [(t(r, "End_Timestamp") - t(r, "Start_Timestamp")) / 1e3 for r in timed]
    gaps = [(t(b, "Start_Timestamp") - t(a, "End_Timestamp")) / 1e3 for a, b in zip(timed, timed[1:])]
    region = (t(sync, "End_Timestamp") - t(ev0, "Start_Timestamp")) / 1e3
    items = {
        "ev0_record_to_first_launch_call_us": (t(launches[0], "Start_Timestamp") - t(ev0, "Start_Timestamp")) / 1e3,
        "first_launch_call_to_first_kernel_start_us": (t(timed[0], "Start_Timestamp") -
                                                        t(launches[0], "Start_Timestamp")) / 1e3,
        "kernels_sum_us": sum(durs),
        "gaps_between_kernels_sum_us": sum(gaps),
        "last_kernel_end_to_sync_return_us": (t(sync, "End_Timestamp") - t(timed[-1], "End_Timestamp")) / 1e3,
    }
    out = {
        "source": "rocprofv3 --kernel-trace --hip-trace -- python3 bench.py --no-cpu --gpus 1 --steps %d --warmup 5" % K,
        "timed_region_us (ev0 record start -> hipDeviceSynchronize return)": round(region, 2),
        "items_us": {k: round(v, 2) for k, v in items.items()},
        "items_sum_check_us": round(sum(items.values()), 2),
        "kernel_us": {"first": round(durs[0], 3), "second": round(durs[1], 3), "mean": round(statistics.mean(durs), 3),
                      "median": round(statistics.median(durs), 3), "mean_without_first": round(statistics.mean(durs[1:]), 3),
                      "all": [round(x, 3) for x in durs]},
        "gap_us": {"mean": round(statistics.mean(gaps), 3), "max": round(max(gaps), 3),
                   "all": [round(x, 3) for x in gaps]},
        "host_launch_call_us": {"first": round((t(launches[0], "End_Timestamp") - t(launches[0], "Start_Timestamp")) / 1e3, 2),
                                "mean": round(statistics.mean((t(r, "End_Timestamp") - t(r, "Start_Timestamp")) / 1e3
                                                              for r in launches), 2),
                                "last_launch_returns_before_last_kernel_start_us":
                                    round((t(timed[-1], "Start_Timestamp") - t(launches[-1], "End_Timestamp")) / 1e3, 2)},
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
