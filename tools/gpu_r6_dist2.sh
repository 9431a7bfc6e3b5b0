# Round 6: the default build's C5 / dist tests, then the A/B of the distance
# path knobs (base = acq_rel arrival + opaque item tid, no part lists; spill =
# round 5's item loop; relaxed = round 5's arrival; pl = part lists on), then
# the PMC profile of the C5 steady state on the default build.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r6/dist2}"; mkdir -p "$OUT"; cd "$R"
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "c5 or dist" \
  > "$OUT/tests_dist.log" 2>&1 || { tail -40 "$OUT/tests_dist.log"; exit 1; }
tail -1 "$OUT/tests_dist.log"
fi
for rep in 1 2; do
  for v in ${VARIANTS:-base spill relaxed pl}; do
    for w in "default 200 20" "steady 30 600"; do
      set -- $w
      MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_$v.so" timeout -k 10 300 python3 bench.py --config c5 --no-cpu \
        --steps $2 --warmup $3 > "$OUT/c5_${1}_${v}_$rep.json" 2> "$OUT/c5_${1}_${v}_$rep.err" || { tail -5 "$OUT/c5_${1}_${v}_$rep.err"; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/c5_${1}_${v}_$rep.json')); print('$1 $v rep $rep', round(d['value']/1e6,2), 'M', d['roofline']['kernel_us'], 'us')"
    done
  done
done
[ -n "${SKIP_PROF:-}" ] && exit 0
timeout -k 10 900 python3 tools/prof_config.py --config c5 --steps 30 --warmup 600 --sq --out "$OUT/prof/c5_steady" > "$OUT/prof_c5.log" 2>&1 || { tail -5 "$OUT/prof_c5.log"; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/prof/c5_steady/summary.json'))
for k, v in d.get('kernels', {}).items(): print(k[:60], {x: v.get(x) for x in ('mean_us', 'hbm_read_bytes_per_step', 'hbm_write_bytes_per_step')})
" || true
exit 0
