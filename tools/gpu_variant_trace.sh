# Per-kernel mean durations of the timed steps for variant libraries:
#   VARIANTS="base cur" ARGS="--config c5 --steps 30 --warmup 600" [TAG=x] bash tools/gpu_variant_trace.sh
# ("cur" = the in-tree libmarlcov.so; "cur:ENV=VAL" runs it with one env var set)
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-vtrace}"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
K=$(echo "$ARGS" | sed -n 's/.*--steps \([0-9]*\).*/\1/p')
for spec in ${VARIANTS}; do
  v=${spec%%:*}; ev=""; [ "$v" != "$spec" ] && ev=${spec#*:}
  lib="$R/marl-coverage_amd/libmarlcov_v_$v.so"; [ "$v" = cur ] && lib="$R/marl-coverage_amd/libmarlcov.so"
  name=$(echo "$spec" | tr ':=' '__')
  ( [ -n "$ev" ] && export "$ev"; export MARLCOV_LIB="$lib"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu $ARGS > "$OUT/$name.log" 2>&1 )
  rc=$?; echo "== $spec rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 - "$OUT/$name/run_kernel_trace.csv" "$K" <<'PY'
import csv, statistics, sys, collections
K = int(sys.argv[2])
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "rocclr" not in r["Kernel_Name"] and "random_actions" not in r["Kernel_Name"]
        and "at::" not in r["Kernel_Name"]]
env = [i for i, r in enumerate(rows) if "env_kernel" in r["Kernel_Name"] or "sg_step" in r["Kernel_Name"]]
first = env[-K]  # the timed steps: from the K-th last env kernel on
d = collections.defaultdict(float)
for r in rows[first:]:
    d[r["Kernel_Name"].split("(")[0][:70]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for k, v in d.items():
    print(f"  {k:70s} {v / K:9.2f} us per step")
span = (int(rows[-1]["End_Timestamp"]) - int(rows[first]["Start_Timestamp"])) / 1e3
print(f"  step total {sum(d.values()) / K:.2f} us (trace span {span / K:.2f} us per step)")
PY
done
exit 0
