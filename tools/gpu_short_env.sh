# The driver's short form (--steps 20 --warmup 5) under HSA / HIP runtime
# settings, alternating, REPS rounds: the host's wait for the last kernel
# (HSA_ENABLE_INTERRUPT=0: signal waits poll instead of sleeping on an
# interrupt) and the kernel-argument placement (HIP_FORCE_DEV_KERNARG=1).
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r5/short_env}"; mkdir -p "$OUT"; cd "$R"
for r in $(seq 1 ${REPS:-4}); do
  for m in default nointr devkarg both; do
    case $m in
      default) E="";;
      nointr) E="HSA_ENABLE_INTERRUPT=0";;
      devkarg) E="HIP_FORCE_DEV_KERNARG=1";;
      both) E="HSA_ENABLE_INTERRUPT=0 HIP_FORCE_DEV_KERNARG=1";;
    esac
    env $E timeout -k 10 120 python3 bench.py --no-cpu --gpus 1 --steps 20 --warmup 5 > "$OUT/k20_${m}_$r.json" 2> "$OUT/k20_${m}_$r.err" || { tail -5 "$OUT/k20_${m}_$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,1), d['ms_per_step']*1e3, d['roofline']['kernel_us'])" "$OUT/k20_${m}_$r.json" "k20 $m $r"
  done
done
