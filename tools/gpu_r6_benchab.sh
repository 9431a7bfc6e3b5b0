# A/B of the grid-baked bench instantiations (base) against the shapes with
# runtime grids (nobench), C2 / C4 / C5 steady, 3 alternating reps; then the
# env-kernel GPU tests on the default build.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r6/benchab}"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "c2 or c4 or c5 or shape or fullsize or shards" \
  > "$OUT/tests.log" 2>&1 || { tail -60 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for rep in 1 2 3; do
  for v in base nobench; do
    for c in "c2 200 20" "c4 50 5" "c5 30 600"; do
      set -- $c
      MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_$v.so" timeout -k 10 300 python3 bench.py --config $1 --no-cpu \
        --steps $2 --warmup $3 > "$OUT/$1_${v}_$rep.json" 2> "$OUT/$1_${v}_$rep.err" || { tail -5 "$OUT/$1_${v}_$rep.err"; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/$1_${v}_$rep.json')); print('$1 $v rep $rep', round(d['value']/1e6,2), 'M', d['roofline']['kernel_us'], 'us', d['config']['kernel_variant'])"
    done
  done
done
exit 0
