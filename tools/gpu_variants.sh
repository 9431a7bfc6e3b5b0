# A/B variants of the bench in one GPU session (kernel-time + wall), plus one PMC pass
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/var
run() { name=$1; shift; timeout -k 10 120 "$@" > gpurun_out/var/$name.json 2> gpurun_out/var/$name.err; rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/var/$name.json | head -1) $(grep -o '"kernel_us": [0-9.]*' gpurun_out/var/$name.json)"; return $rc; }
run base python bench.py --no-cpu || exit 1
run noreset python bench.py --no-cpu --maxsteps 1000000000 || exit 1
MARLCOV_NT=128 run nt128 python bench.py --no-cpu || exit 1
MARLCOV_NT=256 run nt256 python bench.py --no-cpu || exit 1
run envs8k python bench.py --no-cpu --envs 8192 || exit 1
run envs16k python bench.py --no-cpu --envs 16384 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/var/pmc1" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu --steps 50 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/var/pmc1.log" 2>&1
echo "pmc1 rc=$?"
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/var/pmc2" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu --steps 50 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/var/pmc2.log" 2>&1
echo "pmc2 rc=$?"
