# C5 bench line and its per-kernel breakdown (rocprofv3 kernel trace).
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/c5"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 bench.py --no-cpu --config c5 --steps ${STEPS:-20} --warmup ${WARM:-10} > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('c5', round(d['value']/1e6,3), 'M', d['ms_per_step'], 'ms', d['config'].get('dist_full_transforms_last_step'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --config c5 --steps ${STEPS:-20} --warmup ${WARM:-10} > "$OUT/trace.log" 2>&1 || exit 1
cut -d, -f1-4 "$OUT/trace/run_kernel_stats.csv" | cut -c1-150
exit 0
