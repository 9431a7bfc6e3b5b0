set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 180 python bench.py > gpurun_out/bm_graph.json 2> gpurun_out/bm_graph.err || { tail -20 gpurun_out/bm_graph.err; exit 1; }
cat gpurun_out/bm_graph.json
timeout -k 10 120 python bench.py --no-cpu --eager > gpurun_out/bm_eager.json 2> gpurun_out/bm_eager.err || exit 1
grep -o '"value": [0-9.]*\|"kernel_us": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/bm_eager.json | head -3
timeout -k 10 300 python bench.py --no-cpu --config c4 > gpurun_out/bm_c4.json 2> gpurun_out/bm_c4.err || { tail -5 gpurun_out/bm_c4.err; exit 1; }
grep -o '"value": [0-9.]*\|"kernel_us": [0-9.]*\|"ms_per_step": [0-9.]*\|"achieved": [0-9.]*' gpurun_out/bm_c4.json | head -4
