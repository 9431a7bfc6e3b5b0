# Same-box A/B of variant libraries on one bench config, alternating runs:
#   VARIANTS="base new" CONFIG=c4 [STEPS=30 WARMUP=5 REPS=3] bash tools/gpu_ab_config.sh
# (variants: marl-coverage_amd/libmarlcov_v_<name>.so, selected by MARLCOV_LIB)
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/ab_${CONFIG}"; mkdir -p "$OUT"; cd "$R"
for rep in $(seq 1 ${REPS:-3}); do
  for v in ${VARIANTS}; do
    MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_$v.so" timeout -k 10 180 python3 bench.py --no-cpu --config $CONFIG --steps ${STEPS:-30} --warmup ${WARMUP:-5} > "$OUT/${v}_$rep.json" 2> "$OUT/${v}_$rep.err" || exit 1
    python3 -c "import json; d=json.load(open('$OUT/${v}_$rep.json')); print('$v rep $rep', round(d['value']/1e6,3), 'M', d['roofline']['kernel_us'], 'us')"
  done
done
exit 0
