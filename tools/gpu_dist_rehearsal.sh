# Rehearsal of bench.py's multi-rank flow (torchrun, barriers, max-over-ranks
# time, the episode-statistics all-reduce, rank-0 JSON line) on a 1-GPU box:
# two ranks on the same GPU over gloo.  The driver's N > 1 runs use RCCL.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/dist_rehearsal"; mkdir -p "$OUT"
cd "$R"
for cfg in c2 sg_c2; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 --config $cfg --dist-backend gloo \
    > "$OUT/n2_$cfg.json" 2> "$OUT/n2_$cfg.err" || { tail -20 "$OUT/n2_$cfg.err"; exit 1; }
  cat "$OUT/n2_$cfg.json"
done
exit 0
