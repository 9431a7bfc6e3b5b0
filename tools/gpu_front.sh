# GPU parity suite on the default library, then an A/B of variant libraries
# (VARIANTS, tools/build_variants.py) at C2.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/front"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.log"; [ $rc -ne 0 ] && exit $rc
VARIANTS="${VARIANTS}" bash tools/gpu_ab_pair.sh
