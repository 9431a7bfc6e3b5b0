# The driver's short bench form vs the long form on one lease (VERDICT r3
# item 2): --steps 20 --warmup 5 with each launch mode, K = 200, and the
# rocprofv3 kernel mean of the short form.  CONFIG (default c2), REPS (3).
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-short_form}"; mkdir -p "$OUT"; cd "$R"
C=${CONFIG:-c2}
for rep in $(seq 1 ${REPS:-3}); do
  for mode in native stream graph; do
    timeout -k 10 180 python3 bench.py --no-cpu --config $C --steps 20 --warmup 5 --launch $mode > "$OUT/k20_${mode}_$rep.json" 2> "$OUT/k20_${mode}_$rep.err" || exit 1
    python3 -c "import json; d=json.load(open('$OUT/k20_${mode}_$rep.json')); print('K=20 $mode rep $rep', round(d['value']/1e6,2), 'M', d['ms_per_step']*1e3, 'us/step', d['roofline']['kernel_us'], 'kernel_us', d['config']['host_issue_us_per_step'], 'issue_us')"
  done
  timeout -k 10 180 python3 bench.py --no-cpu --config $C --steps 200 --warmup 20 > "$OUT/k200_native_$rep.json" 2> "$OUT/k200_native_$rep.err" || exit 1
  python3 -c "import json; d=json.load(open('$OUT/k200_native_$rep.json')); print('K=200 native rep $rep', round(d['value']/1e6,2), 'M', d['ms_per_step']*1e3, 'us/step', d['roofline']['kernel_us'], 'kernel_us', d['config']['host_issue_us_per_step'], 'issue_us')"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --config $C --steps 20 --warmup 5 > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
cut -d, -f1-8 "$OUT/trace/run_kernel_stats.csv" | head -4
exit 0
