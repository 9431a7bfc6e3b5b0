# dist_reward loop: dist parity tests first, the whole GPU suite, then C5 and C2 benches
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="${TAG:-d}"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread -k "dist or c5" > gpurun_out/${T}_dist_tests.log 2>&1
rc=$?; echo "dist pytest rc=$rc"; tail -3 gpurun_out/${T}_dist_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config c5 --no-cpu --steps ${C5_STEPS:-50} --warmup 5 > gpurun_out/${T}_c5.json 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"kernel_us": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/${T}_c5.json | head -3
timeout -k 10 120 python bench.py --no-cpu > gpurun_out/${T}_c2.json 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"kernel_us": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/${T}_c2.json | head -3
