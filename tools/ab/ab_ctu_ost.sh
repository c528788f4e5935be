#!/bin/bash
# A/B of config 4's output path (NH_CTU_OST: 0 row pieces from registers, 1 luma /
# 2 chroma / 3 both through LDS output images with whole-row stores) on the A/B
# library, alternating processes; one JSON line per run (bench_configs --configs 4b).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${TAG:-ab}
OUT=gpurun_out/ab_ctu_ost_${TAG}.jsonl
for rep in 1 2; do
  for ost in 0 1 2 3; do
    NH_CTU_OST=$ost timeout -k 10 120 python tools/bench_configs.py --ab --configs 4b --reps 20 >> $OUT || exit 1
  done
done
cat $OUT
