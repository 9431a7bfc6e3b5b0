# A/B of launch variants on the C2 bench (graph mode): default, EPW=1
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="${TAG:-ab}"
for v in "default" "MARLCOV_EPW=1"; do
  if [ "$v" = default ]; then envs=""; else envs="$v"; fi
  env $envs timeout -k 10 120 python bench.py --no-cpu > gpurun_out/${T}_${v//=/_}.json 2>&1 || exit 1
  echo "== $v"; grep -o '"value": [0-9.]*\|"kernel_us": [0-9.]*' gpurun_out/${T}_${v//=/_}.json | head -2
  env $envs timeout -k 10 120 python bench.py --no-cpu --envs 16384 > gpurun_out/${T}_${v//=/_}_16k.json 2>&1 || exit 1
  grep -o '"value": [0-9.]*\|"kernel_us": [0-9.]*' gpurun_out/${T}_${v//=/_}_16k.json | head -2
done
