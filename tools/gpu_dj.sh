# dijkstra_input layer: parity (window + full-map modes), the whole GPU suite,
# the c2_dijkstra bench line and its kernel trace.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-dj}"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "dijkstra" --timeout 300 --timeout-method thread > "$OUT/dj_tests.log" 2>&1
rc=$?; tail -5 "$OUT/dj_tests.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --config c2_dijkstra --cpu-secs 2.5 > "$OUT/bench_c2_dijkstra.json" 2> "$OUT/bench.err"
rc=$?; cat "$OUT/bench_c2_dijkstra.json"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --config c2_dijkstra --no-cpu --steps 100 --warmup 300 > "$OUT/bench_c2_dijkstra_w300.json" 2> "$OUT/bench.err"
rc=$?; cat "$OUT/bench_c2_dijkstra_w300.json"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --config c2_dijkstra --no-cpu > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
cut -d, -f1-5 "$OUT/trace/run_kernel_stats.csv" | head -8
exit 0
