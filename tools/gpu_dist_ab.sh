# dist_reward GPU tests first (every -m gpu test whose name mentions dist / c5 /
# C5 / known / fullsize), then the C5 steady / early trace means of VARIANTS.
#   TAG=r5/fused VARIANTS="unfused cur" bash tools/gpu_dist_ab.sh
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-dist_ab}"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -k "dist or c5 or C5 or fullsize" -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
SKIP_TESTS=1 SHAPES="${SHAPES:-c5s c5e}" TAG="${TAG:-dist_ab}" bash tools/gpu_ab_round.sh
