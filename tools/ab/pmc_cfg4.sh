#!/bin/bash
# SQ wave-state PMC pass of the config-4 batched stream (bench_configs --configs 4b) on the
# A/B build, one pass per form: FORMS="NH_CTU_NARROW=0 NH_CTU_NARROW=1" (comma = several knobs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmc4}
CTRS=${CTRS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY"}
i=0
for form in ${FORMS:-"NH_CTU_NARROW=0" "NH_CTU_NARROW=1"}; do
  i=$((i+1))
  echo "== $form"
  env ${form//,/ } timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/${TAG}_$i -o run -- python3 tools/bench_configs.py --ab --configs 4b --reps 3 > gpurun_out/${TAG}_$i.log 2>&1 || exit 1
  echo "$form" > gpurun_out/${TAG}_$i/form.txt
done
