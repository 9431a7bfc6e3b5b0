# rocprofv3 kernel-trace summary of the exact bench command + PMC traffic passes
set -u
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; T="${TAG:-x}"; OUT="$R/gpurun_out/prof_$T"; mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  n=$(echo $grp | cut -d' ' -f1)
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace -d "$OUT/pmc_$n" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --eager --steps 50 --warmup 5 > "$OUT/pmc_$n.log" 2>&1
  rc=$?; echo "pmc $n rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
