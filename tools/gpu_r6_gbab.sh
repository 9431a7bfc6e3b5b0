# Env-kernel A/B: 64-bit row planes gathered by byte loads (gb, the tree)
# against HEAD: the env-kernel GPU tests on gb (lidar ray / fan / square
# paths), then C4 / C2 / C5 steady, 3 alternating reps.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r6/gbab}"; mkdir -p "$OUT"; cd "$R"
MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_gb.so" timeout -k 10 900 python -u -m pytest tests -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "c2 or c4 or c5 or parity or fullsize or fan or lidar" > "$OUT/tests_gb.log" 2>&1 || { tail -40 "$OUT/tests_gb.log"; exit 1; }
tail -1 "$OUT/tests_gb.log"
VARIANTS="head gb" CONFIGS="c4:50:5 c2:200:20 c5:30:600" TAG="${TAG:-r6/gbab}" bash tools/gpu_r6_ab3.sh
