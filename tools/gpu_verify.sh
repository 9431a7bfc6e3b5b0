# Round verification on one MI355X: every GPU test (FIRST=<files> run first),
# smoke(), the default bench line and the rocprofv3 kernel-trace summary of
# that same command.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${VERIFY_TAG:-verify}"; mkdir -p "$OUT"
cd "$R"
if [ -n "${FIRST:-}" ]; then
  timeout -k 10 900 python -u -m pytest $FIRST -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests_first.log" 2>&1
  rc=$?; tail -5 "$OUT/gpu_tests_first.log"; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; tail -2 "$OUT/smoke.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
cat "$OUT/bench_c2.json"
[ -n "${NO_TRACE:-}" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
cut -d, -f1-4 "$OUT/trace/run_kernel_stats.csv" | head -3
exit 0
