# SuperGridRL: GPU parity tests, then the bench line and a kernel-trace summary
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/sg"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_super.py -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --config sg_c2 ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
cat "$OUT/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --config sg_c2 --no-cpu > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
cut -d, -f1-4 "$OUT/trace/run_kernel_stats.csv" | head -4
exit 0
