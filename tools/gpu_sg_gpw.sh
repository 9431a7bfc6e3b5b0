# SuperGridRL step kernel at several envs-per-wave caps (MARLCOV_SG_GPW), sg_c2,
# rocprofv3 kernel trace of each:  GPWS="4 2" bash tools/gpu_sg_gpw.sh
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/sg_gpw"; mkdir -p "$OUT"; cd /tmp; export TMPDIR=/tmp
for g in ${GPWS:-4 2}; do
  MARLCOV_SG_GPW=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/g$g" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --config sg_c2 --steps 50 --warmup 5 > "$OUT/g$g.json" 2> "$OUT/g$g.err" || exit 1
  python3 - "$OUT/g$g/run_kernel_stats.csv" "$g" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "sg_" in r["Name"]:
        print("gpw", sys.argv[2], r["Name"][:48], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done
