set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -rs > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 180 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu --steps 200 --warmup 20 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
echo "prof rc=$?"
