# Round 6, first GPU call: the late-rank shard tests at the bench shapes, the
# bench's own N-rank launcher (2 gloo ranks on the one GPU, no torchrun in the
# command), the default bench line.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/r6_first"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests/test_gpu_reference_maps.py tests/test_gpu_fullsize.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "full_size or bg2" > "$OUT/fullsize.log" 2>&1
rc=$?; tail -8 "$OUT/fullsize.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu \
  > "$OUT/bench_gpus2_gloo.json" 2> "$OUT/bench_gpus2_gloo.err"
rc=$?; echo "launcher rc=$rc"; cat "$OUT/bench_gpus2_gloo.json"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu > "$OUT/bench_gpus2_rccl.json" 2> "$OUT/bench_gpus2_rccl.err"
echo "rccl on one GPU rc=$? (expected non-zero)"; tail -2 "$OUT/bench_gpus2_rccl.err"
timeout -k 10 300 python3 bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench_c2.json"
exit $rc
