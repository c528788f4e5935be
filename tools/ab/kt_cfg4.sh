#!/bin/bash
# Per-kernel times (rocprofv3 --kernel-trace --stats) of the config-4 batched stream on the
# A/B build, one trace per form: FORMS="NH_CTU_T32=2 NH_CTU_T32=0" (comma = several knobs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-kt4}
i=0
for form in ${FORMS:-"NH_CTU_T32=2" "NH_CTU_T32=0"}; do
  i=$((i+1))
  env ${form//,/ } timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_$i -o run -- python3 tools/bench_configs.py --ab --configs 4b --reps 10 > gpurun_out/${TAG}_$i.log 2>&1 || exit 1
  echo "$form" > gpurun_out/${TAG}_$i/form.txt
  echo "== $form"
  grep -h "ctu" gpurun_out/${TAG}_$i/run_kernel_stats.csv | cut -d, -f1-8
done
