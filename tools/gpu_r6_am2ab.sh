# Env-kernel A/B: the POST window search with the passes' first row reads
# issued together (am2, the tree) against HEAD: the C5 / dist GPU tests on
# am2, then C5 steady / default window, 3 alternating reps.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r6/am2ab}"; mkdir -p "$OUT"; cd "$R"
MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_am2.so" timeout -k 10 900 python -u -m pytest tests -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "c5 or dist" > "$OUT/tests_am2.log" 2>&1 || { tail -40 "$OUT/tests_am2.log"; exit 1; }
tail -1 "$OUT/tests_am2.log"
VARIANTS="head am2" CONFIGS="c5:30:600 c5:200:20" TAG="${TAG:-r6/am2ab}" bash tools/gpu_r6_ab3.sh
