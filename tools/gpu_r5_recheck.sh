# Round 5: the dist / C4 / C5 GPU tests, the C4 and C5-steady bench lines and
# their rocprofv3 profiles (traffic + SQ) after a change to those kernels.
#   TAG=r5/final2 bash tools/gpu_r5_recheck.sh
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r5/final2}"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -k "dist or c4 or C4 or c5 or C5 or fullsize or 360 or fan" -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 300 python3 bench.py --config c4 --steps 50 --warmup 5 --no-cpu > "$OUT/bench_c4.json" || exit 1
timeout -k 10 300 python3 bench.py --config c5 --steps 30 --warmup 600 --no-cpu > "$OUT/bench_c5_steady.json" || exit 1
timeout -k 10 900 python3 tools/prof_config.py --config c4 --steps 30 --warmup 5 --sq --out "$OUT/prof/c4" > "$OUT/prof_c4.log" 2>&1 || { tail -5 "$OUT/prof_c4.log"; exit 1; }
timeout -k 10 900 python3 tools/prof_config.py --config c5 --steps 30 --warmup 600 --sq --out "$OUT/prof/c5_steady" > "$OUT/prof_c5.log" 2>&1 || { tail -5 "$OUT/prof_c5.log"; exit 1; }
echo done
