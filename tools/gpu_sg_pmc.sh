# PMC passes (one counter group per run) over the SuperGridRL bench, eager launches
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/sg_pmc"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace -d "$OUT/p$i" -o run --output-format csv -- python3 "$R/bench.py" --config sg_c2 --no-cpu --eager --steps 30 --warmup 5 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pmc $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
