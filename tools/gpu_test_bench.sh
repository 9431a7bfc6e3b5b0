# GPU parity tests + bench + kernel-trace profile (stops at the first GPU failure)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG="${TAG:-run}"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -rs -x > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 180 python bench.py ${BENCH_EXTRA:-} > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu --steps 200 --warmup 20 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" 2>&1
echo "prof rc=$?"
