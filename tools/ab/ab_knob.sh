# A/B of one A/B-library knob on one bench_configs config, alternating processes:
#   TAG=x KNOB=NH_CTU_PLAN VALS="0 1" CFG=4b FIX="NH_CTU_OST=2" bash tools/ab/ab_knob.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
OUT=gpurun_out/ab_${KNOB}_${CFG}_${TAG:-x}.jsonl
for rep in $(seq 1 ${REPS:-2}); do for v in $VALS; do
  echo "{\"knob\": \"$KNOB\", \"val\": \"$v\", \"rep\": $rep, \"fixed\": \"$FIX\"}" >> $OUT
  env $FIX $KNOB=$v timeout -k 10 200 python tools/bench_configs.py --ab --configs $CFG --reps ${BREPS:-20} $BARGS >> $OUT 2>> ${OUT%.jsonl}.err || exit 1
done; done
