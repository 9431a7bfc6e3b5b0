# Round-6 verification and measurement on one lease: every GPU test, smoke(),
# the bench lines (C2 long and the driver's short form x3, C4 and C5 with
# their CPU baselines, C5 steady, SuperGridRL, C2 + dijkstra, the --gpus 2
# launcher rehearsal) and the rocprofv3 profiles of the timed steps (kernel
# trace, FETCH_SIZE / WRITE_SIZE, SQ counters) of C2, C4, C5 steady / default.
#   TAG=r6/final [SKIP_TESTS=1] [SKIP_BENCH=1] [SKIP_PROF=1] bash tools/gpu_r6_final.sh
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r6/final}"; mkdir -p "$OUT"; cd "$R"
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
  tail -1 "$OUT/gpu_tests.log"
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
b() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || { tail -5 "$OUT/bench_$n.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$n.json')); r=d['roofline']; c=d.get('cpu_baseline') or {}; print('$n', round(d['value']/1e6,2), 'M', d['ms_per_step']*1e3, 'us/step', r['kernel_us'], 'kernel_us frac', r['frac'], 'cpu', c.get('value'), c.get('reference_equiv_value'))"
}
if [ -z "${SKIP_BENCH:-}" ]; then
b c2
for i in 1 2 3; do b c2_short_$i --gpus 1 --steps 20 --warmup 5 --no-cpu; done
b c4 --config c4 --steps 50 --warmup 5
b c5_steady --config c5 --steps 30 --warmup 600 --no-cpu
b c5 --config c5
b sg_c2 --config sg_c2 --no-cpu
b c2_dijkstra --config c2_dijkstra --no-cpu
b gpus2_gloo --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu
fi
[ -n "${SKIP_PROF:-}" ] && exit 0
timeout -k 10 900 python3 tools/prof_config.py --config c2 --steps 200 --warmup 20 --sq --out "$OUT/prof/c2" > "$OUT/prof_c2.log" 2>&1 || { tail -5 "$OUT/prof_c2.log"; exit 1; }
timeout -k 10 900 python3 tools/prof_config.py --config c4 --steps 30 --warmup 5 --sq --out "$OUT/prof/c4" > "$OUT/prof_c4.log" 2>&1 || { tail -5 "$OUT/prof_c4.log"; exit 1; }
timeout -k 10 900 python3 tools/prof_config.py --config c5 --steps 30 --warmup 600 --sq --out "$OUT/prof/c5_steady" > "$OUT/prof_c5.log" 2>&1 || { tail -5 "$OUT/prof_c5.log"; exit 1; }
echo prof done
exit 0
