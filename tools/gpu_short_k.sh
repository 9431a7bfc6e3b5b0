# The driver's short form (--steps 20 --warmup 5) and the default, 3 reps each
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/short_k"; mkdir -p "$OUT"
cd "$R"
for rep in 1 2 3; do
  for k in "20 5" "200 20"; do
    set -- $k
    timeout -k 10 120 python3 bench.py --no-cpu --steps $1 --warmup $2 > "$OUT/b_$1_$rep.json" 2> "$OUT/b.err" || exit 1
    python3 -c "import json; d=json.load(open('$OUT/b_$1_$rep.json')); print('K=$1 rep $rep', round(d['value']/1e6,1), 'M', d['ms_per_step']*1e3, 'us wall', d['roofline']['kernel_us'], 'us events')"
  done
done
exit 0
