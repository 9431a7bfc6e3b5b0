# quick loop: GPU parity tests, bench (2 sizes), phase stamps
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="${TAG:-q}"
timeout -k 10 600 python -m pytest tests -m gpu -q -x -rs > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 120 python bench.py --no-cpu > gpurun_out/${T}_bench.json 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"kernel_us": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/${T}_bench.json | head -3
timeout -k 10 120 python bench.py --no-cpu --envs 16384 > gpurun_out/${T}_bench16k.json 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"kernel_us": [0-9.]*' gpurun_out/${T}_bench16k.json | head -2
timeout -k 10 200 python tools/stamps.py > gpurun_out/${T}_stamps.log 2>&1; echo "stamps rc=$?"
cat gpurun_out/${T}_stamps.log | grep -v amdgpu.ids
