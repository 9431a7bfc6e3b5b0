# PMC passes for the env kernel (one counter group per rocprofv3 run; no sys/runtime trace).
set -u
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/pmc"
mkdir -p "$OUT"
ARGS="${BENCH_ARGS:---no-cpu --steps 50 --warmup 5}"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --stats -d "$OUT/p$i" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
