# Round 6: the big-map distance kernel (bg2_1073x1073 with dist_reward) and
# the C5 / dist suite after the opaque thread index in every dist helper;
# then the C5 lines.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r6/big}"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "bg2 or rows_past or c5 or dist or c4" \
  > "$OUT/tests.log" 2>&1 || { tail -60 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for w in "default 200 20" "steady 30 600"; do
  set -- $w
  timeout -k 10 300 python3 bench.py --config c5 --no-cpu --steps $2 --warmup $3 > "$OUT/c5_$1.json" 2> "$OUT/c5_$1.err" || { tail -5 "$OUT/c5_$1.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c5_$1.json')); print('$1', round(d['value']/1e6,2), 'M', d['roofline']['kernel_us'], 'us')"
done
for rep in 1 2; do
  for v in c4base c4w5; do
    MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_$v.so" timeout -k 10 300 python3 bench.py --config c4 --no-cpu \
      --steps 50 --warmup 5 > "$OUT/c4_${v}_$rep.json" 2> "$OUT/c4_${v}_$rep.err" || { tail -5 "$OUT/c4_${v}_$rep.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c4_${v}_$rep.json')); print('c4 $v rep $rep', round(d['value']/1e6,2), 'M', d['roofline']['kernel_us'], 'us', d['config']['kernel_variant'])"
  done
done
exit 0
