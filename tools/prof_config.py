"""Profile one bench.py workload on the GPU box: kernel trace, HBM traffic and
per-wave SQ counters of the TIMED steps only.

    python tools/prof_config.py --config c4 [--steps 50 --warmup 5] [--out gpurun_out/prof_c4]
        [--extra "--maxsteps 2000"] [--sq]

Runs, each in its own process under its own time limit (no --pmc pass is
combined with a trace domain other than --kernel-trace, and every pass holds
at most 8 SQ / 4 TCC counters: MI355X_MICROARCH.md, rocprofv3 PMC slots):
  bench.json        bench.py alone (no profiler)
  trace/            rocprofv3 --kernel-trace --stats
  pmc_fetch/        rocprofv3 --pmc FETCH_SIZE
  pmc_write/        rocprofv3 --pmc WRITE_SIZE
  pmc_sq1/, sq2/    SQ wave-cycle and instruction counters (--sq)
then keeps, per kernel, only the dispatches of the timed region — the last
`steps` dispatches of every kernel that runs once per step — so warm-up and
reset launches do not enter the means, and writes summary.json:
  per kernel: mean / median duration per dispatch (us), dispatches per step,
  HBM bytes per step: read = 2 x FETCH_SIZE (gfx950 counts half of each 128-B
  request, MI355X_MICROARCH.md HBM section), write = WRITE_SIZE; per-wave SQ
  counters; per step: the sums over its kernels.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SQ1 = "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"
SQ2 = "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"


def run(cmd, log, limit):
    print("+", " ".join(cmd), flush=True)
    with open(log, "w") as f:
        r = subprocess.run(["timeout", "-k", "10", str(limit)] + cmd, stdout=f, stderr=subprocess.STDOUT)
    print(f"  rc={r.returncode}", flush=True)
    if r.returncode != 0:
        sys.exit(r.returncode)


def rows(path):
    files = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    return [r for f in files for r in csv.DictReader(open(f))]


def per_dispatch(path):
    """{kernel: [(dispatch id, {counter: value summed over the dispatch})]} in dispatch order."""
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    name = {}
    for r in rows(path):
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        name[d] = r["Kernel_Name"]
    out = collections.defaultdict(list)
    for d in sorted(per):
        out[name[d]].append((d, dict(per[d])))
    return out


def trace(path):
    files = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    out = collections.defaultdict(list)
    for f in files:
        for r in sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"])):
            out[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return out


def short(n):
    return n.split("(")[0][:120]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--extra", default="")
    ap.add_argument("--out", default=None)
    ap.add_argument("--sq", action="store_true")
    ap.add_argument("--limit", type=int, default=240)
    ap.add_argument("--analyze-only", action="store_true", help="re-summarise the runs already under --out")
    args = ap.parse_args()
    out = args.out or os.path.join(ROOT, "gpurun_out", f"prof_{args.config}")
    os.makedirs(out, exist_ok=True)
    bench = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu", "--config", args.config,
             "--steps", str(args.steps), "--warmup", str(args.warmup)] + args.extra.split()
    os.environ.setdefault("TMPDIR", "/tmp")
    passes = [("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")]
    if args.sq:
        passes += [("pmc_sq1", SQ1), ("pmc_sq2", SQ2)]
    if not args.analyze_only:
        run(bench, os.path.join(out, "bench.json"), args.limit)
        prof = ["rocprofv3", "--kernel-trace", "--stats", "-d", os.path.join(out, "trace"), "-o", "run",
                "--output-format", "csv", "--"]
        run(prof + bench, os.path.join(out, "trace.log"), args.limit)
        for d, counters in passes:
            cmd = ["rocprofv3", "--pmc", *counters.split(), "--kernel-trace", "-d", os.path.join(out, d), "-o",
                   "run", "--output-format", "csv", "--"]
            run(cmd + bench, os.path.join(out, d + ".log"), args.limit)
    passes = [p for p in passes if os.path.isdir(os.path.join(out, p[0]))]

    K = args.steps
    tr = trace(os.path.join(out, "trace"))
    summary = {"config": args.config, "steps": K, "warmup": args.warmup, "bench_args": bench[2:], "kernels": {}}
    counters = {}
    for d, _ in passes:
        for k, lst in per_dispatch(os.path.join(out, d)).items():
            counters.setdefault(k, {}).setdefault(d, lst)
    step = collections.defaultdict(float)
    for k, durs in tr.items():
        # a per-step kernel runs in every warmup and timed step; the rest are
        # setup (grids, allocation fills), resets or action staging
        if len(durs) < K + args.warmup or "random_actions" in k or k.startswith("__amd_rocclr"):
            continue
        # dispatches per step (C5's transform kernel runs twice: modes 2 and
        # 3); a reset's extra dispatches do not change the rounding
        m = max(1, round(len(durs) / (K + args.warmup)))
        timed = durs[-K * m:]
        ent = {"dispatches_total": len(durs), "dispatches_per_step": m, "timed_dispatches": K * m,
               "mean_us": round(statistics.mean(timed), 3), "median_us": round(statistics.median(timed), 3),
               "per_step_us": round(statistics.mean(timed) * m, 3)}
        c = counters.get(k, {})
        if "pmc_fetch" in c and "pmc_write" in c:
            # bytes per step: the timed dispatches' sum over K
            f = [x["FETCH_SIZE"] for _, x in c["pmc_fetch"][-K * m:]]
            w = [x["WRITE_SIZE"] for _, x in c["pmc_write"][-K * m:]]
            ent["hbm_read_bytes"] = round(2 * 1024 * sum(f) / K)
            ent["hbm_write_bytes"] = round(1024 * sum(w) / K)
            ent["hbm_bytes"] = ent["hbm_read_bytes"] + ent["hbm_write_bytes"]
            step["hbm_bytes"] += ent["hbm_bytes"]
        sq = {}
        for d in ("pmc_sq1", "pmc_sq2"):
            if d in c:
                lst = c[d][-K * m:]
                for name in lst[0][1]:
                    sq[name] = statistics.median(x[name] for _, x in lst)
        if sq:
            waves = sq.get("SQ_WAVES", 1.0) or 1.0
            ent["sq_median"] = {n: v for n, v in sorted(sq.items())}
            ent["sq_per_wave"] = {n: round(v / waves, 1) for n, v in sorted(sq.items()) if n != "SQ_WAVES"}
        step["mean_us"] += ent["per_step_us"]
        summary["kernels"][short(k)] = ent
    summary["step"] = {k: round(v, 3) for k, v in step.items()}
    with open(os.path.join(out, "summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary["step"]))
    for k, e in summary["kernels"].items():
        print(f"{k[:90]:90s} {e['per_step_us']:10.2f} us  {e.get('hbm_bytes', 0) / 1e6:9.2f} MB per step")


if __name__ == "__main__":
    main()
