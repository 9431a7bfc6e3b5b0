# A/B of library builds (MARLCOV_LIB) on one box: LIBS="name=path ..." for
# each config in CFGS (default c2), ROUNDS alternations to average out drift
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-abl}; mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
for cfg in ${CFGS:-c2}; do
  for lv in $LIBS; do
    n=${lv%%=*}; l=${lv#*=}
    MARLCOV_LIB=$l timeout -k 10 200 python bench.py --no-cpu --config $cfg ${BARGS:-} > $OUT/$n.$cfg.json 2> $OUT/$n.$cfg.err || { cat $OUT/$n.$cfg.err | tail -5; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$n.$cfg.json')); print('r$r $cfg $n', round(d['value']/1e6,2), 'M/s', d['roofline']['kernel_us'], 'us')"
  done
done
done
exit 0
