#!/bin/bash
# Config-4 open-loop launch forms on one box, alternating processes (A/B build):
# NH_CFG4_FORM=1 = round 1's per-size launches; 0 = k_ctu_open with NH_CTU_WAVES = 1 / 3 / 4,
# NH_CTU_T32 = 1 (int8 MFMA) / 0 (butterfly) for the 32x32 TUs.  FORMS="A=1 B=2,C=3" overrides (comma = several knobs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
TAG=${TAG:-ab4}
for rep in 1 2; do
  for form in ${FORMS:-"NH_CFG4_FORM=1" "NH_CTU_WAVES=1" "NH_CTU_WAVES=3" "NH_CTU_WAVES=4"}; do
    env ${form//,/ } timeout -k 10 120 python tools/bench_configs.py --ab --configs 4b --reps 10 >> gpurun_out/ab_cfg4_${TAG}.jsonl 2>> gpurun_out/ab_cfg4_${TAG}.err || exit 1
  done
done
tail -${NTAIL:-8} gpurun_out/ab_cfg4_${TAG}.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['knobs'], round(d['ms_per_frame']*1e3,2), 'us/frame', d['out_digest'])"
