set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/r6/diag"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 400 python3 -u tools/diag_dist_step49.py > "$OUT/diag_step49.txt" 2>&1; rc=$?
cat "$OUT/diag_step49.txt" | tail -40
exit $rc
