# A/B: two envs per wave (default) vs one env per wave (MARLCOV_EPW=1), and
# kernel time vs env count (latency- vs throughput-bound)
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/epw; mkdir -p $OUT
for e in 1024 2048 4096 8192; do
  for epw in 2 1; do
    MARLCOV_EPW=$epw timeout -k 10 120 python bench.py --no-cpu --envs $e > $OUT/e${e}_p${epw}.json 2> $OUT/e${e}_p${epw}.err || exit 1
    python3 -c "import json; d=json.load(open('$OUT/e${e}_p${epw}.json')); print('envs $e epw $epw', round(d['value']/1e6,1), 'M/s', d['roofline']['kernel_us'], 'us')"
  done
done
