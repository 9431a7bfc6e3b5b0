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
K = int(sys.argv[2]); d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    d[r["Kernel_Name"].split("(")[0][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = 0
for k, v in d.items():
    if len(v) > K and "rocclr" not in k and "random_actions" not in k:
        m = statistics.mean(v[-K:]); tot += m; print(f"  {k:70s} {m:9.2f} us")
print(f"  step total {tot:.2f} us")
PY
done
exit 0
