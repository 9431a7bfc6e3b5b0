# A/B of the SuperGridRL step kernel's envs per wave (MARLCOV_SG_GPW), sg_c2.
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; OUT="$R/gpurun_out/${TAG:-sg_gpw}"; mkdir -p "$OUT"
for rep in 1 2; do
  for g in ${GPWS:-1 2 4 8 16}; do
    MARLCOV_SG_GPW=$g timeout -k 10 120 python3 bench.py --no-cpu --config sg_c2 --steps 200 --warmup 20 > "$OUT/g${g}_$rep.json" 2>&1 || exit $?
    python3 -c "import json; s=open('$OUT/g${g}_$rep.json').read(); d=json.loads(s[s.index('{'):]); print('gpw $g rep $rep', round(d['value']/1e6,2), 'M', d['roofline']['kernel_us'], 'us')"
  done
done
cd /tmp && export TMPDIR=/tmp
for g in ${GPWS:-1 2 4 8 16}; do
  MARLCOV_SG_GPW=$g timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace_g$g" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --config sg_c2 --steps 100 --warmup 10 > "$OUT/trace_g$g.log" 2>&1 || exit $?
  grep sg_step "$OUT/trace_g$g/run_kernel_stats.csv" | cut -d, -f1-4
done
exit 0
