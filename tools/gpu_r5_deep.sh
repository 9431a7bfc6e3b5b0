# Round 5: the deep-episode / full-size parity tests, then the dist transform's
# per-part stamps at the C5 steady state and early phase.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r5/deep}"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v --timeout 170 --timeout-method thread --durations=0 > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -12 "$OUT/gpu_tests.log"
timeout -k 10 300 python3 tools/dist_stamps.py --warmup 600 > "$OUT/dstamps_steady.txt" 2>&1 || { tail -5 "$OUT/dstamps_steady.txt"; exit 1; }
cat "$OUT/dstamps_steady.txt"
timeout -k 10 300 python3 tools/dist_stamps.py --warmup 5 > "$OUT/dstamps_early.txt" 2>&1 || { tail -5 "$OUT/dstamps_early.txt"; exit 1; }
cat "$OUT/dstamps_early.txt"
