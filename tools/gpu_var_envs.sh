# Variant libraries x env counts: bench kernel time (stream launches).
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/varenv"; mkdir -p "$OUT"
cd "$R"
for v in ${VARIANTS}; do
  for e in ${ENVS:-2 1024 4096}; do
    MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_$v.so" timeout -k 10 120 python3 bench.py --no-cpu --envs $e > "$OUT/${v}_$e.json" 2> "$OUT/${v}_$e.err" || exit 1
    python3 -c "import json; d=json.load(open('$OUT/${v}_$e.json')); print('$v envs=$e', round(d['value']/1e6,1), 'M', d['roofline']['kernel_us'], 'us')"
  done
done
exit 0
