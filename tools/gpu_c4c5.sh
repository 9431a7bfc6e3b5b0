# C4 and C5 bench lines + kernel-trace summaries
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/c4c5"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for c in c4 c5; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/$c" -o run --output-format csv -- python3 "$R/bench.py" --config $c --no-cpu --steps 60 --warmup 10 > "$OUT/$c.json" 2> "$OUT/$c.err"
  rc=$?; echo "$c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 -c "import json; d=json.load(open('$OUT/$c.json')); print(d['value'], d['ms_per_step'], d['config'].get('dist_full_transforms_last_step'))"
  cut -d, -f1-4 "$OUT/$c/run_kernel_stats.csv" | head -6
done
exit 0
