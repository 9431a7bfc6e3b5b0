# A/B of variant libraries on C2 / C4 / C5 steady, 3 alternating reps:
#   VARIANTS="head udk" bash tools/gpu_r6_ab3.sh
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r6/ab3}"; mkdir -p "$OUT"; cd "$R"
for rep in 1 2 3; do
  for v in ${VARIANTS:-head udk}; do
    for c in ${CONFIGS:-"c2:200:20" "c4:50:5" "c5:30:600"}; do
      IFS=: read -r cf k w <<< "$c"
      MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_$v.so" timeout -k 10 300 python3 bench.py --config $cf --no-cpu \
        --steps $k --warmup $w > "$OUT/${cf}w${w}_${v}_$rep.json" 2> "$OUT/${cf}w${w}_${v}_$rep.err" || { tail -5 "$OUT/${cf}w${w}_${v}_$rep.err"; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/${cf}w${w}_${v}_$rep.json')); print('$cf w$w $v rep $rep', round(d['value']/1e6,2), 'M', d['roofline']['kernel_us'], 'us')"
    done
  done
done
exit 0
