# Distance-path A/B: base (sc1 hand-off, idle parts skip staging), noskip
# (every part stages), plainho (plain hand-off stores / loads under the acq_rel
# arrival): the C5 / dist tests on base and plainho first, then C5 steady /
# default window, 3 alternating reps.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r6/hoab}"; mkdir -p "$OUT"; cd "$R"
for v in base plainho; do
  MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_$v.so" timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v \
    --timeout 300 --timeout-method thread -k "c5 or dist" > "$OUT/tests_$v.log" 2>&1 || { tail -40 "$OUT/tests_$v.log"; exit 1; }
  tail -1 "$OUT/tests_$v.log"
done
VARIANTS="base noskip plainho" CONFIGS="c5:30:600 c5:200:20" TAG="${TAG:-r6/hoab}" bash tools/gpu_r6_ab3.sh
