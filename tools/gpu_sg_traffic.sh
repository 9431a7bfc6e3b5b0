# SuperGridRL HBM bytes per step: separate FETCH_SIZE / WRITE_SIZE passes (eager launches)
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/sg_traffic"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace -d "$OUT/$grp" -o run --output-format csv -- python3 "$R/bench.py" --config sg_c2 --no-cpu --eager --steps 200 --warmup 20 > "$OUT/$grp.log" 2>&1
  rc=$?; echo "pmc $grp rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
