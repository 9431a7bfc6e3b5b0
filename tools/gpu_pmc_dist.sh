# PMC passes for the C5 kernels (one counter group per rocprofv3 run)
set -u
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/pmcd_${TAG:-x}"; mkdir -p "$OUT"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace -d "$OUT/p$i" -o run --output-format csv -- python3 "$R/bench.py" --config c5 --no-cpu --eager --steps 6 --warmup 2 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
