# HEAD verification on one MI355X: every GPU test, smoke(), the default bench
# line (with the CPU baseline), the driver's short form, the rocprofv3
# kernel-trace summary of the default command, and the c2_dijkstra line.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-final}"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -2 "$OUT/gpu_tests.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; tail -2 "$OUT/smoke.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
rc=$?; cat "$OUT/bench_c2.json"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu > "$OUT/bench_c2_short.json" 2> "$OUT/bench.err"
rc=$?; cat "$OUT/bench_c2_short.json"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --config c2_dijkstra --no-cpu > "$OUT/bench_c2_dijkstra.json" 2> "$OUT/bench.err"
rc=$?; cat "$OUT/bench_c2_dijkstra.json"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
cut -d, -f1-4 "$OUT/trace/run_kernel_stats.csv" | head -3
exit 0
