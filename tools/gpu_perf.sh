# parity tests, then C2 (4096 / 16384 envs) and C4 bench lines, then stamps
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="${TAG:-p}"
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/${T}_tests.log
[ $rc -ne 0 ] && exit $rc
for a in "c2" "c2 --envs 16384" "c4" "c5" "c2_dijkstra"; do
  n=${a// /_}
  timeout -k 10 200 python bench.py --no-cpu --config $a > gpurun_out/${T}_bench_$n.json 2>&1 || exit 1
  echo "== $a: $(grep -o '"value": [0-9.]*\|"kernel_us": [0-9.]*' gpurun_out/${T}_bench_$n.json | head -2 | tr '\n' ' ')"
done
if [ -n "${STAMPS:-}" ]; then
  timeout -k 10 200 python tools/stamps.py > gpurun_out/${T}_stamps.log 2>&1 || exit 1
  grep -E "rt|stage|sense|whole|merge|moves|store|obs |eager" gpurun_out/${T}_stamps.log
fi
exit 0
