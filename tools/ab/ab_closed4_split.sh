#!/bin/bash
# Config-4 closed loop A/B with split timing (tools/ab/ab_closed4_split.py), alternating processes.
#   RUNS="--lib:tools/_ab/libnanohevc_head.so --lib:nano-hevc_amd/nano_hevc/libnanohevc.so --ab:NH_CLOSED4_MULTI_C=1" \
#   TAG=x REPS=3 tools/ab/ab_closed4_split.sh
# A run is "--lib:PATH", "--ab:KNOB=V,KNOB=V" or "product".
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
TAG=${TAG:-split}
OUT=gpurun_out/ab_closed4_split_${TAG}.jsonl
for rep in $(seq ${REPS:-3}); do
  for run in $RUNS; do
    case "$run" in
      --lib:*) env timeout -k 10 150 python tools/ab/ab_closed4_split.py --lib "${run#--lib:}" $ARGS >> $OUT || exit 1 ;;
      --ab:*)  kv="${run#--ab:}"; env ${kv//,/ } timeout -k 10 150 python tools/ab/ab_closed4_split.py --ab $ARGS >> $OUT || exit 1 ;;
      *)       timeout -k 10 150 python tools/ab/ab_closed4_split.py $ARGS >> $OUT || exit 1 ;;
    esac
  done
done
python3 - "$OUT" <<'EOF'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["lib"], d["knobs"], *(f"{k} {d[k]['median_ms_per_frame']:.4f}" for k in d if isinstance(d[k], dict) and "median_ms_per_frame" in d[k]), d["out_digest"])
EOF
