# A/B of k_tc32_hd's block order / blocks per wave on the compact levels (A/B library knobs)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
OUT=gpurun_out/ab_tc32_${TAG:-x}.jsonl
for rep in 1 2; do for cfg in ${CFGS:-"2 2" "0 2"}; do
  set -- $cfg
  echo "{\"ilv\": $1, \"kb\": $2, \"rep\": $rep}" >> $OUT
  NH_TC32H_ILV=$1 NH_TC32H_DMA=$2 timeout -k 10 200 python tools/bench_configs.py --ab --configs 5b --cfg5-levels ${LEVELS:-int32,int16,int8} --reps 20 >> $OUT 2>> ${OUT%.jsonl}.err || exit 1
done; done
