# HBM traffic of the C2 env kernel: separate --pmc passes for FETCH_SIZE and
# WRITE_SIZE (MI355X_MICROARCH.md HBM/rocprofv3 section), plus one SQ pass.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TRAFFIC_TAG:-traffic}"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmc_$c" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --steps 20 --warmup 5 ${BENCH_ARGS:-} > "$OUT/pmc_$c.log" 2>&1 || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_LDS --kernel-trace -d "$OUT/pmc_sq" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --steps 20 --warmup 5 ${BENCH_ARGS:-} > "$OUT/pmc_sq.log" 2>&1 || exit 1
exit 0
