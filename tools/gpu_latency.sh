# Latency floor of the C2 step: bench at small env counts, and phase stamps
# (stamped build) at 1024 and 4096 envs.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/lat"; mkdir -p "$OUT"
cd "$R"
for e in 2 256 1024; do
  timeout -k 10 120 python3 bench.py --no-cpu --envs $e > "$OUT/e$e.json" 2>&1 || exit 1
  python3 -c "import json; s=open('$OUT/e$e.json').read(); d=json.loads(s[s.index('{'):]); print('envs $e', d['ms_per_step']*1e3, d['roofline']['kernel_us'])"
done
for e in 1024 4096; do
  timeout -k 10 200 python3 tools/stamps.py --envs $e > "$OUT/stamps_$e.log" 2>&1 || exit 1
done
exit 0
