# Distance-path A/B: the strips' carries from per-row word masks (rwm, the
# tree) against HEAD: the C5 / dist / reference-map GPU tests on rwm, then C5
# steady / default window, 3 alternating reps.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r6/rwmab}"; mkdir -p "$OUT"; cd "$R"
MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_rwm.so" timeout -k 10 900 python -u -m pytest tests -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "c5 or dist or reference_maps" > "$OUT/tests_rwm.log" 2>&1 || { tail -40 "$OUT/tests_rwm.log"; exit 1; }
tail -1 "$OUT/tests_rwm.log"
VARIANTS="head rwm" CONFIGS="c5:30:600 c5:200:20" TAG="${TAG:-r6/rwmab}" bash tools/gpu_r6_ab3.sh
