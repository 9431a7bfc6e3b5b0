# Round 5 measurement items on one lease: FETCH_SIZE calibration (VERDICT r4
# item 6), the driver's short form traced with HIP API timestamps and the
# host-sync A/B (item 7), and the 2-rank gloo rehearsal of the multi-rank bench
# at HEAD (item 8).
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r5/misc}"; mkdir -p "$OUT"; cd "$R"
[ -n "${SKIP_FETCH:-}" ] || TAG="${TAG:-r5/misc}/fetch" bash tools/gpu_fetch_calib.sh > "$OUT/fetch.log" 2>&1 || { tail -5 "$OUT/fetch.log"; exit 1; }
[ -n "${SKIP_FETCH:-}" ] || tail -3 "$OUT/fetch.log"
for rep in 1 2 3; do
  for s in default spin; do
    timeout -k 10 180 python3 bench.py --no-cpu --steps 20 --warmup 5 --sync $s > "$OUT/k20_${s}_$rep.json" 2> "$OUT/k20_${s}_$rep.err" || exit 1
  done
  timeout -k 10 180 python3 bench.py --no-cpu --steps 200 --warmup 20 > "$OUT/k200_default_$rep.json" 2> "$OUT/k200_$rep.err" || exit 1
done
python3 -c "
import json,glob
for f in sorted(glob.glob('$OUT/k*.json')):
    d=json.load(open(f)); print(f.split('/')[-1], round(d['value']/1e6,1), d['ms_per_step']*1e3, d['roofline']['kernel_us'])"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 50 --warmup 5 > "$OUT/dist_rehearsal.json" 2> "$OUT/dist_rehearsal.err" || { tail -5 "$OUT/dist_rehearsal.err"; exit 1; }
cat "$OUT/dist_rehearsal.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --hip-trace -d "$OUT/trace_hip" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --gpus 1 --steps 20 --warmup 5 > "$OUT/trace_hip.log" 2>&1 || { tail -5 "$OUT/trace_hip.log"; exit 1; }
timeout -k 10 180 rocprofv3 --kernel-trace --hip-trace -d "$OUT/trace_hip_spin" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --gpus 1 --steps 20 --warmup 5 --sync spin > "$OUT/trace_hip_spin.log" 2>&1 || { tail -5 "$OUT/trace_hip_spin.log"; exit 1; }
ls "$OUT/trace_hip"
exit 0
