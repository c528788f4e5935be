#!/bin/bash
# hipExtMallocWithFlags contiguous vs default backing, several processes each (tools/ab_hipalloc.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01as}
for f in 4 0 4 0 4 0; do
  timeout -k 10 120 python tools/ab_hipalloc.py --flags $f >> gpurun_out/ab_hipalloc_${TAG}.jsonl 2>>gpurun_out/ab_hipalloc_${TAG}.err || exit 1
  tail -1 gpurun_out/ab_hipalloc_${TAG}.jsonl
done
echo "== done"
