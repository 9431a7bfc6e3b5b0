# A/B of variant libraries (tools/build_variants.py) at C2, alternating runs:
#   VARIANTS="base nt" [EXTRA="HIP_FORCE_DEV_KERNARG=1"] bash tools/gpu_ab_pair.sh
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/abpair"; mkdir -p "$OUT"
cd "$R"
for rep in 1 2 3; do
  for v in ${VARIANTS}; do
    for k in "200 20" "20 5"; do
      set -- $k
      MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_$v.so" timeout -k 10 120 python3 bench.py --no-cpu --steps $1 --warmup $2 > "$OUT/${v}_$1_$rep.json" 2> "$OUT/${v}_$1_$rep.err" || exit 1
      python3 -c "import json; d=json.load(open('$OUT/${v}_$1_$rep.json')); print('$v K=$1 rep $rep', round(d['value']/1e6,1), 'M', d['roofline']['kernel_us'], 'us')"
    done
  done
done
if [ -n "${EXTRA:-}" ]; then
  for rep in 1 2; do
    env $EXTRA MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_base.so" timeout -k 10 120 python3 bench.py --no-cpu > "$OUT/extra_$rep.json" 2>&1 || exit 1
    python3 -c "import json; s=open('$OUT/extra_$rep.json').read(); d=json.loads(s[s.index('{'):]); print('base+$EXTRA', round(d['value']/1e6,1), 'M', d['roofline']['kernel_us'], 'us')"
  done
fi
exit 0
