# C5 moves A/B (round 5): parity of the fixed-point moves (moves_par) on the
# C5 shape, then per-kernel trace means of the serial-moves variant
# (libmarlcov_v_serial.so, -DMC_MOVES_SERIAL=1) against the in-tree build at
# the steady and early phases, and phase stamps of both (stamped variants).
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r5/c5moves}"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shapes.py tests/test_gpu_fullsize.py -k "c5 or C5" -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
VARIANTS="${VARIANTS:-serial cur}" ARGS="--config c5 --steps 30 --warmup 600" TAG="${TAG:-r5/c5moves}/steady" bash tools/gpu_variant_trace.sh || exit 1
VARIANTS="${VARIANTS:-serial cur}" ARGS="--config c5 --steps 30 --warmup 5" TAG="${TAG:-r5/c5moves}/early" bash tools/gpu_variant_trace.sh || exit 1
for v in ${STAMPS:-stamps stampser}; do
  timeout -k 10 300 python3 tools/stamps.py --config c5 --envs 8192 --lib "$R/marl-coverage_amd/libmarlcov_v_$v.so" > "$OUT/stamps_$v.txt" 2>&1 || { tail -5 "$OUT/stamps_$v.txt"; exit 1; }
  grep -E "moves|merge|whole|eager" "$OUT/stamps_$v.txt"
done
exit 0
