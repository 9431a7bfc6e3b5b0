# For each variant library: bench (stream launches) + one PMC pass of SQ
# instruction counts with kernel trace.  VARIANTS="base abl1 ..." (built by
# tools/build_variants.py).
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/pmcvar"; mkdir -p "$OUT"
cd "$R"
for v in ${VARIANTS}; do
  lib="$R/marl-coverage_amd/libmarlcov_v_$v.so"
  MARLCOV_LIB=$lib timeout -k 10 120 python3 bench.py --no-cpu ${BENCH_ARGS:-} > "$OUT/$v.json" 2> "$OUT/$v.err" || exit 1
  python3 -c "import json; d=json.load(open('$OUT/$v.json')); print('$v', round(d['value']/1e6,1), 'M', d['roofline']['kernel_us'], 'us')"
  if [ -n "${PMC:-1}" ]; then
    ( cd /tmp && export TMPDIR=/tmp && MARLCOV_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_LDS --kernel-trace -d "$OUT/pmc_$v" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --steps 20 --warmup 5 ${BENCH_ARGS:-} > "$OUT/pmc_$v.log" 2>&1 ) || exit 1
  fi
done
exit 0
