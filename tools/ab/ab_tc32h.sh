#!/bin/bash
# A/B of config 5's f16 kernel forms (NH_TC32H_FORM: 0 plain, 1 XCD-ordered grid,
# 2 whole-row output stores, 3 both) on the A/B library, alternating processes,
# plus the product library; one JSON line per run (bench_configs --configs 5b).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${TAG:-ab}
OUT=gpurun_out/ab_tc32h_${TAG}.jsonl
for rep in 1 2; do
  for form in 0 1 2 3; do
    NH_TC32H_FORM=$form timeout -k 10 120 python tools/bench_configs.py --ab --configs 5b --reps 20 >> $OUT || exit 1
  done
  timeout -k 10 120 python tools/bench_configs.py --configs 5b --reps 20 | sed 's/^{/{"lib": "product", /' >> $OUT || exit 1
done
cat $OUT
