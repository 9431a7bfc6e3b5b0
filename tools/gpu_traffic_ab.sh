# bench + FETCH/WRITE PMC passes for variant libraries
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/traf"; mkdir -p "$OUT"
cd "$R"
for v in ${VARIANTS}; do
  lib="$R/marl-coverage_amd/libmarlcov_v_$v.so"
  MARLCOV_LIB=$lib timeout -k 10 120 python3 bench.py --no-cpu ${BENCH_ARGS:-} > "$OUT/$v.json" 2> "$OUT/$v.err" || exit 1
  python3 -c "import json; d=json.load(open('$OUT/$v.json')); print('$v', round(d['value']/1e6,1), 'M', d['roofline']['kernel_us'], 'us')"
  for c in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && export TMPDIR=/tmp && MARLCOV_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmc_${v}_$c" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --steps 20 --warmup 5 ${BENCH_ARGS:-} > "$OUT/pmc_${v}_$c.log" 2>&1 ) || exit 1
  done
done
exit 0
