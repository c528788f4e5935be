# A/B of environment settings (A/B-library knobs) on one bench_configs config, alternating processes:
#   TAG=x CFG=5b ENVS="NH_X=0|NH_X=1 NH_Y=2" BARGS="--cfg5-levels int16" bash tools/ab/ab_env.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
OUT=gpurun_out/ab_env_${CFG}_${TAG:-x}.jsonl
IFS='|' read -r -a SETS <<< "$ENVS"
for rep in $(seq 1 ${REPS:-2}); do for e in "${SETS[@]}"; do
  echo "{\"env\": \"$e\", \"rep\": $rep}" >> $OUT
  env $e timeout -k 10 200 python tools/bench_configs.py --ab --configs $CFG --reps ${BREPS:-20} $BARGS >> $OUT 2>> ${OUT%.jsonl}.err || exit 1
done; done
