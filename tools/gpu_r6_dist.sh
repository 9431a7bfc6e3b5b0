# Round 6: the C5 distance path after the acq_rel arrival, the threshold
# clamp and the part lists.  1) the C5 / dist GPU tests on the default build
# (incl. the auto-reset split-map oracle test and the totals bookkeeping);
# 2) the split/unsplit identity with the separate-merge build (MC_DIST_FUSED=0);
# 3) C5 early (default window) and steady A/B: base / relaxed arrival / no part
# lists / both (round 5's path), two alternating reps.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r6/dist}"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "c5 or dist" \
  > "$OUT/tests_dist.log" 2>&1 || { tail -40 "$OUT/tests_dist.log"; exit 1; }
tail -1 "$OUT/tests_dist.log"
MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_fused0.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_shapes.py \
  -m gpu -x -v --timeout 300 --timeout-method thread -k "unsplit or auto_reset_match" > "$OUT/tests_fused0.log" 2>&1 \
  || { tail -40 "$OUT/tests_fused0.log"; exit 1; }
tail -1 "$OUT/tests_fused0.log"
[ -n "${SKIP_AB:-}" ] && exit 0
for rep in 1 2; do
  for v in ${VARIANTS:-base relaxed nopl old}; do
    for w in "default 200 20" "steady 30 600"; do
      set -- $w
      MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_$v.so" timeout -k 10 300 python3 bench.py --config c5 --no-cpu \
        --steps $2 --warmup $3 > "$OUT/c5_${1}_${v}_$rep.json" 2> "$OUT/c5_${1}_${v}_$rep.err" || { tail -5 "$OUT/c5_${1}_${v}_$rep.err"; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/c5_${1}_${v}_$rep.json')); print('$1 $v rep $rep', round(d['value']/1e6,2), 'M', d['roofline']['kernel_us'], 'us')"
    done
  done
done
exit 0
