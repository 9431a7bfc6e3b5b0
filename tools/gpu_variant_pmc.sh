# Per-variant kernel time and LDS / wave counters on one bench config:
#   VARIANTS="base abl1 ..." CONFIG=c4 bash tools/gpu_variant_pmc.sh
# (marl-coverage_amd/libmarlcov_v_<name>.so, selected by MARLCOV_LIB).  One
# rocprofv3 --pmc pass per variant (SQ block only), kernel trace included.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-vpmc}_${CONFIG}"; mkdir -p "$OUT"
ARGS="--no-cpu --config $CONFIG --steps ${STEPS:-30} --warmup ${WARMUP:-5}"
CTRS="${CTRS:-SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES}"
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS}; do
  MARLCOV_LIB="$R/marl-coverage_amd/libmarlcov_v_$v.so" timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-trace -d "$OUT/$v/p1" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/$v.log" 2>&1
  rc=$?; echo "== $v rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  python3 "$R/tools/pmc_summary.py" "$OUT/$v" "${KERNEL:-env_kernel}" | grep -E "LDS|WAVE|VALU|WAIT|BUSY"
  python3 - "$OUT/$v/p1/run_kernel_trace.csv" "${KERNEL:-env_kernel}" <<'PY'
import csv, statistics, sys
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r["Kernel_Name"]]
print(f"kernel mean {statistics.mean(d[-30:]):.2f} us median {statistics.median(d[-30:]):.2f} us over {len(d[-30:])}")
PY
done
exit 0
