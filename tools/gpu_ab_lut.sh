set -u
R="$GRAFT_REPO_ROOT"; cd "$R"
MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_lutt.so" timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fan or C4 or c4 or lidar360" > gpurun_out/lutt_tests.log 2>&1; rc=$?; tail -2 gpurun_out/lutt_tests.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="base lutt" CONFIG=c4 REPS=3 bash tools/gpu_ab_config.sh
