# Env-kernel A/B: the State re-read at phase boundaries (rl1, MC_RELOAD=1) vs
# one State for the whole kernel (rl0): the env-kernel GPU tests on rl1, then
# C2 / C4 / C5 steady / C5 default window, 3 alternating reps.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r6/rlab}"; mkdir -p "$OUT"; cd "$R"
MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_rl1.so" timeout -k 10 900 python -u -m pytest tests -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "c2 or c4 or c5 or parity or fullsize" > "$OUT/tests_rl1.log" 2>&1 || { tail -40 "$OUT/tests_rl1.log"; exit 1; }
tail -1 "$OUT/tests_rl1.log"
VARIANTS="rl0 rl1" CONFIGS="c2:200:20 c4:50:5 c5:30:600 c5:200:20" TAG="${TAG:-r6/rlab}" bash tools/gpu_r6_ab3.sh
