# Same-box A/B of variant libraries on any bench arguments, alternating runs:
#   VARIANTS="base cur" ARGS="--config c5 --steps 30 --warmup 600" [REPS=2 TAG=x] bash tools/gpu_ab_bench.sh
# (variants: marl-coverage_amd/libmarlcov_v_<name>.so; "cur" = the in-tree libmarlcov.so)
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-ab_bench}"; mkdir -p "$OUT"; cd "$R"
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS}; do
    lib="$R/marl-coverage_amd/libmarlcov_v_$v.so"; [ "$v" = cur ] && lib="$R/marl-coverage_amd/libmarlcov.so"
    MARLCOV_LIB="$lib" timeout -k 10 300 python3 bench.py --no-cpu $ARGS > "$OUT/${v}_$rep.json" 2> "$OUT/${v}_$rep.err" || exit 1
    python3 -c "import json; d=json.load(open('$OUT/${v}_$rep.json')); print('$v rep $rep', round(d['value']/1e6,3), 'M', d['roofline']['kernel_us'], 'us', d['config'].get('dist_listed_maps_last_step',''), d['config'].get('dist_cache_served_last_step',''))"
  done
done
exit 0
