# Change check: GPU tests, then C2 and C4 bench lines (kernel time).
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/ab"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:-} > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.log"; [ $rc -ne 0 ] && exit $rc
for cfg in c2 c4; do
  timeout -k 10 300 python3 bench.py --no-cpu --config $cfg > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || exit 1
  python3 -c "import json; d=json.load(open('$OUT/bench_$cfg.json')); print('$cfg', round(d['value']/1e6,2), 'M', d['roofline']['kernel_us'], 'us')"
done
exit 0
