#!/bin/bash
# Allocation-order cases for the hot kernel, one process each (tools/ab_alloc.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01ar}
for c in ${CASES:-adjacent gap4 gap2 gap1 outfirst pre2 pre8 adjacent gap4}; do
  timeout -k 10 120 python tools/ab_alloc.py --case $c >> gpurun_out/ab_alloc_${TAG}.jsonl 2>>gpurun_out/ab_alloc_${TAG}.err || exit 1
  tail -1 gpurun_out/ab_alloc_${TAG}.jsonl
done
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True timeout -k 10 120 python tools/ab_alloc.py --case adjacent >> gpurun_out/ab_alloc_${TAG}.jsonl 2>>gpurun_out/ab_alloc_${TAG}.err || exit 1
tail -1 gpurun_out/ab_alloc_${TAG}.jsonl
echo "== done"
