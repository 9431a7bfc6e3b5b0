# GPU parity suite, then C2 bench (default and with env overrides from AB_ENVS,
# e.g. AB_ENVS="MARLCOV_NO_K1=1"), then C4
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-tab}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
for v in "" ${AB_ENVS:-}; do
  env $v timeout -k 10 120 python bench.py --no-cpu > $OUT/b.json 2> $OUT/b.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/b.json')); print('c2 [$v]', round(d['value']/1e6,1), 'M/s', d['roofline']['kernel_us'], 'us')"
done
timeout -k 10 200 python bench.py --no-cpu --config c4 --steps 50 --warmup 5 > $OUT/c4.json 2> $OUT/c4.err || exit 1
python3 -c "import json; d=json.load(open('$OUT/c4.json')); print('c4', round(d['value']/1e6,2), 'M/s', d['roofline']['kernel_us'], 'us')"
exit 0
