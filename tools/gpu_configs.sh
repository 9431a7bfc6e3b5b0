# bench lines of the other BASELINE configs (C4, C5) and the SURVEY 8(f)
# SuperGridRL workload at HEAD, with rocprof kernel summaries for C4 / C5
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-configs}"; mkdir -p "$OUT"
cd "$R"
for cfg in c4 c5 sg_c2; do
  timeout -k 10 300 python3 bench.py --config $cfg --no-cpu --steps 50 --warmup 5 > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || exit 1
  python3 -c "import json; d=json.load(open('$OUT/bench_$cfg.json')); print('$cfg', round(d['value']/1e6,2), 'M', d['roofline']['kernel_us'], 'us', d['roofline']['frac'])"
done
cd /tmp && export TMPDIR=/tmp
for cfg in c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$cfg" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --no-cpu --steps 50 --warmup 5 > "$OUT/trace_$cfg.log" 2>&1 || exit 1
  python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/trace_$cfg/run_kernel_stats.csv')))[:5]: print('$cfg', r['Name'][:60], r['Calls'], r['AverageNs'], r['Percentage'])"
done
exit 0
