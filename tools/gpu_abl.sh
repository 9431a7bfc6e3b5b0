# Diagnostic ablations (tools/build_variants.py a1..a5: -DMC_ABL=k, results
# wrong by design) timed on the C5 steady / C4 bench shapes, plus the dist
# transform's part timeline stamps.
set -u
R="$GRAFT_REPO_ROOT"; T="${TAG:-r5/abl}"; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 300 python3 tools/dist_stamps.py --warmup 600 > "$OUT/dstamps_tl.txt" 2>&1 || { tail -5 "$OUT/dstamps_tl.txt"; exit 1; }
grep -E "parts|timeline|merged|stage split" "$OUT/dstamps_tl.txt"
VARIANTS="cur a1 a2 a3 a4 a5" ARGS="--config c5 --steps 30 --warmup 600" TAG="$T/c5s" bash tools/gpu_variant_trace.sh 2>&1 | grep -E "==|env_kernel" || exit 1
VARIANTS="cur a4 a5" ARGS="--config c4 --steps 30 --warmup 5" TAG="$T/c4" bash tools/gpu_variant_trace.sh 2>&1 | grep -E "==|env_kernel" || exit 1
