# A/B: the cache-try kernel's State / arguments re-read per map (fr) and, on
# top, per-part candidate segments without the returning atomic (seg, the
# tree), against the tree before both (base = one-pass staging + the
# transform's re-reads): the C5 / dist GPU tests on seg, then C5 steady /
# default window / early steps, 3 alternating reps.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r6/frab}"; mkdir -p "$OUT"; cd "$R"
MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_seg.so" timeout -k 10 900 python -u -m pytest tests -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "c5 or dist or reference_maps" > "$OUT/tests_seg.log" 2>&1 || { tail -40 "$OUT/tests_seg.log"; exit 1; }
tail -1 "$OUT/tests_seg.log"
VARIANTS="base fr seg" CONFIGS="c5:30:600 c5:200:20 c5:20:5" TAG="${TAG:-r6/frab}" bash tools/gpu_r6_ab3.sh
