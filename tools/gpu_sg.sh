# SuperGridRL workload: bench line, rocprofv3 kernel-trace summary, HBM PMC passes
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/sg"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 bench.py --config sg_c2 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
cat "$OUT/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --config sg_c2 --no-cpu > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace -d "$OUT/pmc_$grp" -o run --output-format csv -- python3 "$R/bench.py" --config sg_c2 --no-cpu --eager --steps 50 --warmup 5 > "$OUT/pmc_$grp.log" 2>&1
  rc=$?; echo "pmc $grp rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
