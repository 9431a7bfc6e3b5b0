# Full GPU suite, then per-kernel trace means of VARIANTS (default "prev cur")
# on the C5 steady / C5 early / C4 / C2 bench shapes, and C5 stamps of STAMPS.
#   TAG=r5/ab1 [VARIANTS="prev cur"] [SKIP_TESTS=1] [SHAPES="c5s c5e c4 c2"] bash tools/gpu_ab_round.sh
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-ab}"; mkdir -p "$OUT"; cd "$R"
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
  tail -2 "$OUT/gpu_tests.log"
fi
for sh in ${SHAPES:-c5s c5e c4 c2}; do
  case $sh in
    c5s) A="--config c5 --steps 30 --warmup 600";;
    c5e) A="--config c5 --steps 30 --warmup 5";;
    c4) A="--config c4 --steps 30 --warmup 5";;
    c2) A="--config c2 --steps 200 --warmup 20";;
  esac
  echo "== $sh: $A"
  VARIANTS="${VARIANTS:-prev cur}" ARGS="$A" TAG="${TAG:-ab}/$sh" bash tools/gpu_variant_trace.sh || exit 1
done
for v in ${STAMPS:-}; do
  timeout -k 10 300 python3 tools/stamps.py --config c5 --envs 8192 --lib "$R/marl-coverage_amd/libmarlcov_v_$v.so" > "$OUT/stamps_$v.txt" 2>&1 || { tail -5 "$OUT/stamps_$v.txt"; exit 1; }
  grep -E "rt1|moves|merge|reward|obs|whole|eager" "$OUT/stamps_$v.txt"
done
exit 0
