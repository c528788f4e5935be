#!/bin/bash
# Config 5's LDS-DMA form (k_tc32_hd, NH_TC32H_DMA = blocks per wave): parity
# against the product kernel (tc32hd_check.py), then the timing A/B on the A/B
# library (0 = the kept form), alternating processes, two passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${TAG:-ab}
OUT=gpurun_out/ab_tc32hd_${TAG}.jsonl
for kb in 2 4 8; do
  NH_TC32H_DMA=$kb timeout -k 10 180 python tools/ab/tc32hd_check.py >> $OUT || exit 1
done
for rep in 1 2; do
  for kb in 0 2 4 8; do
    NH_TC32H_DMA=$kb timeout -k 10 120 python tools/bench_configs.py --ab --configs 5b --reps 20 | sed "s/^{/{\"dma\": $kb, /" >> $OUT || exit 1
  done
done
cat $OUT
