# parity tests + bench, then phase stamps of the stamped build and ablations
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="${TAG:-q}"
timeout -k 10 600 python -m pytest tests -m gpu -q -x -rs > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python bench.py --no-cpu > gpurun_out/${T}_bench.json 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"kernel_us": [0-9.]*' gpurun_out/${T}_bench.json | head -2
timeout -k 10 120 python bench.py --no-cpu --envs 16384 > gpurun_out/${T}_bench16k.json 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"kernel_us": [0-9.]*' gpurun_out/${T}_bench16k.json | head -2
exec_abl="${ABL:-1 3}"
for a in "" $exec_abl; do
  if [ -z "$a" ]; then arg=""; n=base; else arg="--abl $a"; n=abl$a; fi
  timeout -k 10 200 python tools/stamps.py $arg > gpurun_out/${T}_stamps_$n.log 2>&1 || exit 1
  echo "== $n"; grep -E "rt|stage|sense|whole|merge|moves|store|obs |eager" gpurun_out/${T}_stamps_$n.log
done
