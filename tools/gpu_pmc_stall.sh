# Where a C2 wave's time goes: wave-parked (s_waitcnt / barrier) vs issue
# stall vs active, per instruction type; LDS array cycles and conflicts.
# SQ_* cycle counters count quad-cycles (MI355X_MICROARCH.md).
set -u
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/pmcstall${TAG:-}"
mkdir -p "$OUT"
ARGS="${BENCH_ARGS:---no-cpu --steps 50 --warmup 5}"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d "$OUT/p$i" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 "$R/tools/pmc_summary.py" "$OUT"
exit 0
