# The driver's short form (--steps 20 --warmup 5) under the timed region's
# event placements (--events around / after-first / none) and the stream
# launch, alternating, REPS rounds; one K = 200 line per event placement.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r5/short_events}"; mkdir -p "$OUT"; cd "$R"
for r in $(seq 1 ${REPS:-4}); do
  for m in around after-first none stream; do
    if [ $m = stream ]; then A="--launch stream"; else A="--events $m"; fi
    timeout -k 10 120 python3 bench.py --no-cpu --gpus 1 --steps 20 --warmup 5 $A > "$OUT/k20_${m}_$r.json" 2> "$OUT/k20_${m}_$r.err" || { tail -5 "$OUT/k20_${m}_$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,1), d['ms_per_step']*1e3, d['roofline']['kernel_us'], d['config']['host_issue_us_per_step'])" "$OUT/k20_${m}_$r.json" "k20 $m $r"
  done
done
for m in around after-first; do
  timeout -k 10 120 python3 bench.py --no-cpu --gpus 1 --steps 200 --warmup 20 --events $m > "$OUT/k200_$m.json" 2> "$OUT/k200_$m.err" || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,1), d['ms_per_step']*1e3, d['roofline']['kernel_us'])" "$OUT/k200_$m.json" "k200 $m"
done
