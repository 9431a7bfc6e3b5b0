"""Join tools/micro/fetch_probe's known byte counts with its rocprofv3
FETCH_SIZE / WRITE_SIZE passes (tools/gpu_fetch_calib.sh): bytes per count
unit for each access shape.

    python3 tools/fetch_calib.py <dir with known.json, pmc_FETCH_SIZE/, pmc_WRITE_SIZE/>
"""
import csv
import glob
import json
import os
import sys


def dispatches(d, counter):
    rows = []
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] == counter:
                    rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    return [(k, v) for _, k, v in rows if not k.startswith(("flush", "__amd"))]


def durations(d):
    """Kernel durations (us) in dispatch order, flush / runtime kernels left out."""
    rows = []
    for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"],
                             (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    rows.sort()
    return [t for _, k, t in rows if not k.startswith(("flush", "__amd"))]


def main(d):
    known = json.load(open(os.path.join(d, "known.json")))
    order = known["order"]
    out = {"source": "tools/micro/fetch_probe.hip (known byte counts) + rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                     "passes; the second of two dispatches of each shape, each after a 1 GiB flush",
           "shapes": {}}
    for counter, key in (("FETCH_SIZE", "read"), ("WRITE_SIZE", "write")):
        ds = dispatches(os.path.join(d, "pmc_" + counter), counter)
        us = durations(os.path.join(d, "pmc_" + counter))
        assert len(ds) == 2 * len(order) == len(us), (counter, len(ds), len(us))
        for name, (kname, kb), t in zip(order, ds[len(order):], us[len(order):]):
            if (key == "read") == name.startswith("w_"):
                continue
            b = kb * 1024
            lines = known["lines_touched"][name]
            used = known[key + "_bytes_used"][name]
            out["shapes"][name] = {"kernel": kname.split("(")[0], "counter": counter, "counter_bytes": round(b),
                                   "lines_touched": lines, "line_bytes": lines * 128, "bytes_used": used,
                                   "counter_over_line_bytes": round(b / (lines * 128), 4),
                                   "line_bytes_over_counter": round(lines * 128 / b, 4) if b else None,
                                   "kernel_us": round(t, 1),
                                   "line_bytes_per_s_TBps": round(lines * 128 / (t * 1e-6) / 1e12, 2)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
