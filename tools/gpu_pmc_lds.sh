# LDS PMC passes for the env kernel: wave-time split and LDS array cycles / conflicts.
set -u
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/${PMC_TAG:-pmclds}"
mkdir -p "$OUT"
ARGS="${BENCH_ARGS:---no-cpu --steps 50 --warmup 5}"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU" \
           "SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --stats -d "$OUT/p$i" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 "$R/tools/pmc_summary.py" "$OUT"
exit 0
