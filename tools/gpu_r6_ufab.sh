# Env-kernel A/B: the env's flags uniform (readfirstlane; read back from LDS
# after the step's branch) and its counters re-read before the sensing (uf,
# the tree) against HEAD (head): the env-kernel GPU tests on uf, then C2 / C4
# / C5 steady / C5 default window, 3 alternating reps.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r6/ufab}"; mkdir -p "$OUT"; cd "$R"
MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_uf.so" timeout -k 10 900 python -u -m pytest tests -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "c2 or c4 or c5 or parity or fullsize or episodes" > "$OUT/tests_uf.log" 2>&1 || { tail -40 "$OUT/tests_uf.log"; exit 1; }
tail -1 "$OUT/tests_uf.log"
VARIANTS="head uf" CONFIGS="c2:200:20 c4:50:5 c5:30:600 c5:200:20" TAG="${TAG:-r6/ufab}" bash tools/gpu_r6_ab3.sh
