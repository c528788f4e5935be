#!/bin/bash
# Generic A/B of one NH_* knob of the A/B library over a bench_configs config,
# alternating processes, REPS rounds:   KNOB=NH_TC32H_K VALUES="1 2" CFG=5b TAG=x tools/ab/ab_knob.sh
# (EXTRA: more environment assignments for every run, e.g. EXTRA="NH_TC32H_CAP=2")
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${TAG:-ab}
REPS=${REPS:-2}
OUT=gpurun_out/ab_${KNOB}_${CFG}_${TAG}.jsonl
for rep in $(seq $REPS); do
  for v in $VALUES; do
    env $EXTRA $KNOB=$v timeout -k 10 120 python tools/bench_configs.py --ab --configs $CFG --reps 20 >> $OUT || exit 1
  done
done
cat $OUT
