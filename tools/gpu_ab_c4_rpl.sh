# C4 A/B of beams per lane (EPW = 1 builds): RPL 2 (base) vs 3
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/ab_c4_rpl"; mkdir -p "$OUT"
cd "$R"
for rep in 1 2; do
  for v in base rpl3; do
    MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_$v.so" timeout -k 10 200 python3 bench.py --config c4 --no-cpu --steps 50 --warmup 5 > "$OUT/${v}_$rep.json" 2> "$OUT/${v}_$rep.err" || exit 1
    python3 -c "import json; d=json.load(open('$OUT/${v}_$rep.json')); print('$v rep $rep', round(d['value']/1e6,2), 'M', d['roofline']['kernel_us'], 'us')"
  done
done
exit 0
