# Distance-path A/B: one-pass staging into the extended bitboard (s1) and
# the State / arguments re-read at the item's phase boundaries (rl), both
# (s1rl, the tree), against HEAD's library (head): the C5 / dist GPU tests
# on s1rl first, then C5 steady / default window, 3 alternating reps.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r6/s1ab}"; mkdir -p "$OUT"; cd "$R"
MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_s1rl.so" timeout -k 10 900 python -u -m pytest tests -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "c5 or dist or reference_maps" > "$OUT/tests_s1rl.log" 2>&1 || { tail -40 "$OUT/tests_s1rl.log"; exit 1; }
tail -1 "$OUT/tests_s1rl.log"
VARIANTS="head s1 rl s1rl" CONFIGS="c5:30:600 c5:200:20" TAG="${TAG:-r6/s1ab}" bash tools/gpu_r6_ab3.sh
