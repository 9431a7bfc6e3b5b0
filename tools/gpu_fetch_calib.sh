# FETCH_SIZE / WRITE_SIZE calibration (tools/micro/fetch_probe.hip): one
# --pmc pass per counter, then tools/fetch_calib.py joins the known byte counts.
#   TAG=r5/fetch bash tools/gpu_fetch_calib.sh
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-fetch}"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmc_$c" -o run --output-format csv -- "$R/tools/micro/fetch_probe" "$OUT/known.json" > "$OUT/pmc_$c.log" 2>&1 || exit 1
done
python3 "$R/tools/fetch_calib.py" "$OUT" > "$OUT/fetch_calib.json" || exit 1
cat "$OUT/fetch_calib.json"
