# C2 change check: DecGridRL GPU parity, then bench + kernel-trace summary
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/c2ab"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -2 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --no-cpu > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; [ $rc -ne 0 ] && exit $rc
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['kernel_us'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu > "$OUT/trace.log" 2>&1
rc=$?; [ $rc -ne 0 ] && exit $rc
grep env_kernel "$OUT/trace/run_kernel_stats.csv" | awk -F'",' '{print $2}' | cut -d, -f1-4
exit 0
