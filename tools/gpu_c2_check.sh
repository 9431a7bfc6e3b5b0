# smoke + the default bench (C2) + kernel-trace summary of the same command
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/c2"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; cat "$OUT/smoke.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
cat "$OUT/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
cut -d, -f1-4 "$OUT/trace/run_kernel_stats.csv" | head -3
exit 0
