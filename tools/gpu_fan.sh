# Fan-march check on one MI355X: the dense-beam parity cases (sector march and
# ray march), then C4 bench lines (REPS alternating runs, sector march).
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-fan}"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "${K:-fan or C4 or c4 or lidar360}" > "$OUT/tests.log" 2>&1
rc=$?; tail -4 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
for rep in $(seq 1 ${REPS:-2}); do
  timeout -k 10 180 python3 bench.py --no-cpu --config ${CONFIG:-c4} --steps 30 --warmup 5 > "$OUT/bench_$rep.json" 2> "$OUT/bench_$rep.err" || exit 1
  python3 -c "import json; d=json.load(open('$OUT/bench_$rep.json')); print(round(d['value']/1e6,3), 'M', d['roofline']['kernel_us'], 'us', d['config']['kernel_variant'])"
done
exit 0
