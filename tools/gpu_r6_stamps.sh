# Phase stamps at HEAD: env kernel (C5 steady / early, C4, C2) and the C5
# distance path (steady, early).  Diagnostic builds; stamps perturb the
# schedule: read shares.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r6/stamps}"; mkdir -p "$OUT"; cd "$R"
L="$R/marl-coverage_amd/libmarlcov_v_stamps.so"
timeout -k 10 300 python3 tools/stamps.py --lib "$L" --config c5 --envs 8192 --steps 600 > "$OUT/env_c5_steady.txt" 2>&1 || { tail -20 "$OUT/env_c5_steady.txt"; exit 1; }
timeout -k 10 300 python3 tools/stamps.py --lib "$L" --config c5 --envs 8192 --steps 25 > "$OUT/env_c5_early.txt" 2>&1 || exit 1
timeout -k 10 300 python3 tools/stamps.py --lib "$L" --config c4 --envs 8192 --steps 30 > "$OUT/env_c4.txt" 2>&1 || exit 1
timeout -k 10 300 python3 tools/stamps.py --lib "$L" --config c2 --envs 4096 --steps 30 > "$OUT/env_c2.txt" 2>&1 || exit 1
timeout -k 10 300 python3 tools/dist_stamps.py --envs 8192 --warmup 600 > "$OUT/dist_steady.txt" 2>&1 || { tail -20 "$OUT/dist_steady.txt"; exit 1; }
timeout -k 10 300 python3 tools/dist_stamps.py --envs 8192 --warmup 5 > "$OUT/dist_early.txt" 2>&1 || exit 1
for f in "$OUT"/*.txt; do echo "== $f"; grep -v amdgpu.ids "$f" | head -40; done
