# C4 A/B of variant libraries, alternating: VARIANTS="c4base c4grid" bash tools/gpu_r6_c4ab.sh
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r6/c4ab}"; mkdir -p "$OUT"; cd "$R"
for rep in 1 2 3; do
  for v in ${VARIANTS:-c4base c4grid}; do
    MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_$v.so" timeout -k 10 300 python3 bench.py --config c4 --no-cpu \
      --steps 50 --warmup 5 > "$OUT/c4_${v}_$rep.json" 2> "$OUT/c4_${v}_$rep.err" || { tail -5 "$OUT/c4_${v}_$rep.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c4_${v}_$rep.json')); print('c4 $v rep $rep', round(d['value']/1e6,2), 'M', d['roofline']['kernel_us'], 'us', d['config']['kernel_variant'])"
  done
done
exit 0
