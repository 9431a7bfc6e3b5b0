# SuperGridRL step-kernel timing ablations (results invalid by design): kernel-trace per variant
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/sg_abl"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for a in 0 1 2 4 7; do
  MARLCOV_SG_ABL=$a timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/a$a" -o run --output-format csv -- python3 "$R/bench.py" --config sg_c2 --no-cpu --steps 100 > "$OUT/a$a.log" 2>&1
  rc=$?; echo "abl $a rc=$rc"; [ $rc -ne 0 ] && exit $rc
  grep step_kernel "$OUT/a$a/run_kernel_stats.csv" | awk -F'",' '{print $2}' | cut -d, -f1-4
done
exit 0
