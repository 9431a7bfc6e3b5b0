# C5 check: the C5-shaped parity case, then the C5 bench (steady state) with a kernel trace.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/c5ab"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "c5 or dist" > "$OUT/tests.log" 2>&1
rc=$?; tail -2 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --config c5 --steps 20 --warmup 300 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' "$OUT/bench.json"
cut -d, -f1-4 "$OUT/trace/run_kernel_stats.csv" | head -5 | cut -c1-120
exit 0
