# Per-config profiles of the timed steps (tools/prof_config.py): kernel trace,
# FETCH_SIZE / WRITE_SIZE traffic and (SQ=1) per-wave SQ counters.
#   CONFIGS="c2 c4 c5" TAG=r3_prof [SQ=1] [STEADY=600] bash tools/gpu_prof_round.sh
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"
OUT="$R/gpurun_out/${TAG:-prof}"; mkdir -p "$OUT"
SQF=""; [ -n "${SQ:-}" ] && SQF="--sq"
for c in ${CONFIGS:-c2 c4 c5}; do
  timeout -k 10 900 python3 tools/prof_config.py --config $c --steps ${STEPS:-30} --warmup ${WARMUP:-5} $SQF --out "$OUT/$c" || exit $?
done
if [ -n "${STEADY:-}" ]; then
  timeout -k 10 900 python3 tools/prof_config.py --config c5 --steps ${STEPS:-30} --warmup $STEADY --out "$OUT/c5_steady" || exit $?
fi
exit 0
