# extra PMC passes: instruction fetch, LDS waits, TA/TCP occupancy and L2 latency
set -u
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; T="${TAG:-x}"; OUT="$R/gpurun_out/prof_$T"; mkdir -p "$OUT"
i=0
for grp in "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_INSTS_BRANCH" \
           "SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_LDS_ATOMIC SQ_INSTS_SMEM" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" \
           "TA_BUSY_avr TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TA_DATA_STALL_CYCLES_sum" \
           "SQ_BUSY_CYCLES SQ_LEVEL_WAVES SQ_INSTS_VSKIPPED SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace -d "$OUT/pmx_$i" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --eager --steps 50 --warmup 5 > "$OUT/pmx_$i.log" 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
