# Change check on one MI355X: every GPU test, then the C2 bench (stream
# launches, default K/W) and its env-kernel time under rocprofv3.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/ab"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:-} > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --no-cpu > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('C2', round(d['value']/1e6,1), 'M', d['ms_per_step']*1e3, d['roofline']['kernel_us'])"
timeout -k 10 300 python3 bench.py --no-cpu --steps 20 --warmup 5 > "$OUT/bench20.json" 2> "$OUT/bench20.err" || exit 1
python3 -c "import json; d=json.load(open('$OUT/bench20.json')); print('C2 K=20', round(d['value']/1e6,1), 'M', d['ms_per_step']*1e3, d['roofline']['kernel_us'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu > "$OUT/trace.log" 2>&1 || exit 1
grep env_kernel "$OUT/trace/run_kernel_stats.csv" | awk -F'",' '{print $2}' | cut -d, -f1-4
exit 0
