# dijkstra_input: fraction of paths beyond k BFS layers in the c2_dijkstra
# bench (MARLCOV_DJ_DEPTH=k lists them for the full-map kernel)
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/dj_depth"; mkdir -p "$OUT"
cd "$R"
for d in 24 15 12 8 5; do
  MARLCOV_DJ_DEPTH=$d timeout -k 10 300 python3 bench.py --config c2_dijkstra --no-cpu > "$OUT/b_$d.json" 2> "$OUT/b.err" || exit 1
  python3 -c "import json; d=json.load(open('$OUT/b_$d.json')); print('depth $d', d['value'], d['roofline']['kernel_us'], d['config']['dijkstra_full_map_paths_last_step'])"
done
for k in 1000 100; do
  timeout -k 10 300 python3 bench.py --config c2_dijkstra --no-cpu --steps $k --warmup 300 > "$OUT/b_w$k.json" 2> "$OUT/b.err" || exit 1
  python3 -c "import json; d=json.load(open('$OUT/b_w$k.json')); print('warm $k', d['value'], d['roofline']['kernel_us'], d['config']['dijkstra_full_map_paths_last_step'])"
done
exit 0
