cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread -k "dist or c5" > gpurun_out/e1_dist_tests.log 2>&1; rc=$?; tail -3 gpurun_out/e1_dist_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/dist_micro.py 2048 2>&1 | grep reset
timeout -k 10 300 python bench.py --config c5 --no-cpu --steps 50 --warmup 5 > gpurun_out/e1_c5.json 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"dist_full[^,]*' gpurun_out/e1_c5.json
