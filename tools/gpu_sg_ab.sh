# SuperGridRL: parity tests, then the bench with region-only dist writes and with full rewrites
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/sg"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_super.py -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -2 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
MARLCOV_SG_FULL_DIST=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_super.py -x -q --timeout 300 --timeout-method thread > "$OUT/tests_full.log" 2>&1
rc=$?; tail -2 "$OUT/tests_full.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --config sg_c2 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
cat "$OUT/bench.json"
MARLCOV_SG_FULL_DIST=1 timeout -k 10 300 python3 bench.py --config sg_c2 --no-cpu > "$OUT/bench_fulldist.json" 2> "$OUT/bench_fulldist.err"
rc=$?; echo "bench full rc=$rc"; [ $rc -ne 0 ] && exit $rc
cat "$OUT/bench_fulldist.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --config sg_c2 --no-cpu > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
cut -d, -f1-4 "$OUT/trace/run_kernel_stats.csv" | head -3
exit 0
