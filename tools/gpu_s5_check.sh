# Session check: all GPU tests, smoke, the bench in the driver's short form
# and the default form, and the first-launch probe of a short timed region.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-s5}"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; tail -2 "$OUT/smoke.log"; [ $rc -ne 0 ] && exit $rc
for args in "--steps 20 --warmup 5" "" "--steps 20 --warmup 5"; do
  timeout -k 10 300 python3 bench.py --no-cpu $args > "$OUT/b.json" 2> "$OUT/b.err" || exit 1
  python3 -c "import json; d=json.load(open('$OUT/b.json')); print('$args', d['value'], d['ms_per_step'], d['roofline']['kernel_us'])"
done
timeout -k 10 300 python3 tools/first_kernels.py > "$OUT/first.log" 2>&1 || exit 1
cat "$OUT/first.log"
exit 0
