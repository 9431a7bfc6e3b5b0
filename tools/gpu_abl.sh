# phase stamps of the stamped build and of each MC_ABL timing ablation
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for a in "" 1 2 3 4 5; do
  if [ -z "$a" ]; then arg=""; n=base; else arg="--abl $a"; n=abl$a; fi
  timeout -k 10 200 python tools/stamps.py $arg > gpurun_out/stamps_$n.log 2>&1 || exit 1
  echo "== $n"; grep -E "sense|whole|merge|moves|obs |eager" gpurun_out/stamps_$n.log
done
