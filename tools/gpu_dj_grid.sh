# dijkstra_input: A/B of the full-map kernel's fixed grid (c2_dijkstra bench)
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/dj_grid"; mkdir -p "$OUT"
cd "$R"
for g in 256 64 16 256 64 16; do
  MARLCOV_DJ_FULL_GRID=$g timeout -k 10 300 python3 bench.py --config c2_dijkstra --no-cpu > "$OUT/b_$g.json" 2> "$OUT/b.err" || exit 1
  python3 -c "import json; d=json.load(open('$OUT/b_$g.json')); print('grid $g', d['value'], d['roofline']['kernel_us'])"
done
exit 0
