#!/bin/bash
# Config-4 closed-loop forms on one box, alternating processes (A/B build):
# FORMS="NH_TU_CLOSED_PAIR=0 NH_TU_CLOSED_PAIR=1" (comma = several knobs); ARGS: extra bench_configs args.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
TAG=${TAG:-abc4}
for rep in 1 2; do
  for form in ${FORMS:-"NH_TU_CLOSED_PAIR=0" "NH_TU_CLOSED_PAIR=1"}; do
    env ${form//,/ } timeout -k 10 180 python tools/bench_configs.py --ab --configs closed4 --reps 5 $ARGS >> gpurun_out/ab_closed4_${TAG}.jsonl 2>> gpurun_out/ab_closed4_${TAG}.err || exit 1
  done
done
cat gpurun_out/ab_closed4_${TAG}.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d.get('knobs'), d.get('frames'), round(d['ms_per_frame'],4), 'ms/frame', d.get('out_digest', ''))"
