# L2 behaviour of the C2 env kernel: TCC hit/miss and request counts (one
# pass), plus the no-auto-reset bench (reset path cost on the tail).
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/l2"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 120 python3 bench.py --no-cpu --maxsteps 1000000000 > "$OUT/noreset.json" 2>&1 || exit 1
python3 -c "import json; d=json.load(open('$OUT/noreset.json')); print('noreset', d['value'], d['roofline']['kernel_us'])"
timeout -k 10 120 python3 bench.py --no-cpu --envs 1024 > "$OUT/e1024.json" 2>&1 || exit 1
python3 -c "import json; d=json.load(open('$OUT/e1024.json')); print('envs1024', d['value'], d['roofline']['kernel_us'])"
timeout -k 10 120 python3 bench.py --no-cpu --envs 2048 > "$OUT/e2048.json" 2>&1 || exit 1
python3 -c "import json; d=json.load(open('$OUT/e2048.json')); print('envs2048', d['value'], d['roofline']['kernel_us'])"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --kernel-trace -d "$OUT/pmc_tcc" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --steps 20 --warmup 5 > "$OUT/pmc_tcc.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS --kernel-trace -d "$OUT/pmc_sq" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --steps 20 --warmup 5 > "$OUT/pmc_sq.log" 2>&1 || exit 1
exit 0
