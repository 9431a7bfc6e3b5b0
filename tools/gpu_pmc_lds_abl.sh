# LDS conflict share by phase: the LDS counter pass on the default library
# and on timing-ablation variants (MC_ABL=1 marks to the sink only, 3 no sense)
set -u
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-front abl1 abl3}; do
  OUT="$R/gpurun_out/pmclds/$v"; mkdir -p "$OUT"
  MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_$v.so" timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES --kernel-trace -d "$OUT/p1" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --steps 50 --warmup 5 > "$OUT/p1.log" 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 "$R/tools/pmc_summary.py" "$OUT" | grep -v "^kernel"
done
exit 0
