# dist tests, A/B prev vs cur on C5 steady / early, dist part stamps
set -u
R="$GRAFT_REPO_ROOT"; T="${TAG:-r5/stage16}"; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shapes.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -k "c5 or dist" -x -v --timeout 170 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
SKIP_TESTS=1 TAG="$T" VARIANTS="${VARIANTS:-prev cur}" SHAPES="${SHAPES:-c5s c5e}" bash tools/gpu_ab_round.sh || exit 1
timeout -k 10 300 python3 tools/dist_stamps.py --warmup 600 > "$OUT/dstamps_steady.txt" 2>&1 || { tail -5 "$OUT/dstamps_steady.txt"; exit 1; }
grep -E "parts|strips run|stage split|merged" "$OUT/dstamps_steady.txt"
